// Microbenchmark (diagnostic tool): per-SIMD throughput of single VALU instructions on gfx950,
// 16 independent instructions per loop body (inline asm), 1/2/4 waves per SIMD, wall time.
#include <hip/hip_runtime.h>
#include <stdio.h>

#define B2(INS, POST) asm volatile(INS " %0, %0" POST "\n" INS " %1, %1" POST "\n" INS " %2, %2" POST "\n" INS " %3, %3" POST "\n" INS " %4, %4" POST "\n" INS " %5, %5" POST "\n" INS " %6, %6" POST "\n" INS " %7, %7" POST "\n" INS " %8, %8" POST "\n" INS " %9, %9" POST "\n" INS " %10, %10" POST "\n" INS " %11, %11" POST "\n" INS " %12, %12" POST "\n" INS " %13, %13" POST "\n" INS " %14, %14" POST "\n" INS " %15, %15" POST "\n" : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7]), "+v"(r[8]), "+v"(r[9]), "+v"(r[10]), "+v"(r[11]), "+v"(r[12]), "+v"(r[13]), "+v"(r[14]), "+v"(r[15]))
#define B3(INS, POST) asm volatile(INS " %0, %0, %0" POST "\n" INS " %1, %1, %1" POST "\n" INS " %2, %2, %2" POST "\n" INS " %3, %3, %3" POST "\n" INS " %4, %4, %4" POST "\n" INS " %5, %5, %5" POST "\n" INS " %6, %6, %6" POST "\n" INS " %7, %7, %7" POST "\n" INS " %8, %8, %8" POST "\n" INS " %9, %9, %9" POST "\n" INS " %10, %10, %10" POST "\n" INS " %11, %11, %11" POST "\n" INS " %12, %12, %12" POST "\n" INS " %13, %13, %13" POST "\n" INS " %14, %14, %14" POST "\n" INS " %15, %15, %15" POST "\n" : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7]), "+v"(r[8]), "+v"(r[9]), "+v"(r[10]), "+v"(r[11]), "+v"(r[12]), "+v"(r[13]), "+v"(r[14]), "+v"(r[15]))
#define B4(INS, POST) asm volatile(INS " %0, %0, %0, %0" POST "\n" INS " %1, %1, %1, %1" POST "\n" INS " %2, %2, %2, %2" POST "\n" INS " %3, %3, %3, %3" POST "\n" INS " %4, %4, %4, %4" POST "\n" INS " %5, %5, %5, %5" POST "\n" INS " %6, %6, %6, %6" POST "\n" INS " %7, %7, %7, %7" POST "\n" INS " %8, %8, %8, %8" POST "\n" INS " %9, %9, %9, %9" POST "\n" INS " %10, %10, %10, %10" POST "\n" INS " %11, %11, %11, %11" POST "\n" INS " %12, %12, %12, %12" POST "\n" INS " %13, %13, %13, %13" POST "\n" INS " %14, %14, %14, %14" POST "\n" INS " %15, %15, %15, %15" POST "\n" : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7]), "+v"(r[8]), "+v"(r[9]), "+v"(r[10]), "+v"(r[11]), "+v"(r[12]), "+v"(r[13]), "+v"(r[14]), "+v"(r[15]))
template <int MODE>
__global__ void kern(unsigned* out, int iters) {
  unsigned r[16];
  for (int i = 0; i < 16; ++i) r[i] = 0x3c003c00u ^ (threadIdx.x * 7 + i);
  for (int it = 0; it < iters; ++it) {
    if (MODE == 0) B2("v_exp_f32", "");
    if (MODE == 1) B2("v_exp_f16", "");
    if (MODE == 2) B2("v_exp_f16_sdwa", " dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1");
    if (MODE == 3) B3("v_cvt_pk_bf16_f32", "");
    if (MODE == 4) B3("v_cvt_pkrtz_f16_f32", "");
    if (MODE == 5) B4("v_pk_fma_f16", "");
    if (MODE == 6) B3("v_add_f32", "");
    if (MODE == 7) B3("v_pk_add_f16", "");
    if (MODE == 8) B2("v_exp_legacy_f32", "");
  }
  unsigned s = 0;
  for (int i = 0; i < 16; ++i) s ^= r[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int MODE>
void run(const char* name) {
  for (int threads : {128, 256, 512}) {
    const int blocks = 512, iters = 4000;
    unsigned* out;
    (void)hipMalloc(&out, blocks * threads * 4);
    kern<MODE><<<blocks, threads>>>(out, iters);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0), (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    kern<MODE><<<blocks, threads>>>(out, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double wps = (double)blocks * threads / 64 / 1024;
    const double per = ms * 1e-3 / (iters * 16 * wps) * 2.0e9;  // cycles at 2.0 GHz per wave-instruction per SIMD
    printf("%-26s waves/SIMD %.0f: %5.2f cyc/instr/SIMD (at 2.0 GHz)\n", name, wps, per);
    (void)hipFree(out);
  }
}

int main() {
  run<0>("v_exp_f32");
  run<1>("v_exp_f16");
  run<2>("v_exp_f16 sdwa hi");
  run<8>("v_exp_legacy_f32");
  run<3>("v_cvt_pk_bf16_f32");
  run<4>("v_cvt_pkrtz_f16_f32");
  run<5>("v_pk_fma_f16");
  run<7>("v_pk_add_f16");
  run<6>("v_add_f32");
  return 0;
}
