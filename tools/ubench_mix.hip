// Microbenchmark (diagnostic tool): does v_exp_f32 / v_cvt_pk_bf16_f32 issue overlap
// v_mfma_f32_32x32x16_bf16 on one gfx950 SIMD?  Loop body = NM independent-chain MFMAs +
// NE exps (+ NC cvt_pk), cycles per body per SIMD at 1/2/4 waves per SIMD (2.0 GHz basis).
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef __attribute__((__vector_size__(16 * sizeof(float)))) float f32x16;
typedef __attribute__((__vector_size__(8 * sizeof(__bf16)))) __bf16 bf16x8;

#define E16 asm volatile("v_exp_f32 %0, %0\nv_exp_f32 %1, %1\nv_exp_f32 %2, %2\nv_exp_f32 %3, %3\nv_exp_f32 %4, %4\nv_exp_f32 %5, %5\nv_exp_f32 %6, %6\nv_exp_f32 %7, %7\nv_exp_f32 %8, %8\nv_exp_f32 %9, %9\nv_exp_f32 %10, %10\nv_exp_f32 %11, %11\nv_exp_f32 %12, %12\nv_exp_f32 %13, %13\nv_exp_f32 %14, %14\nv_exp_f32 %15, %15\n" : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7]), "+v"(r[8]), "+v"(r[9]), "+v"(r[10]), "+v"(r[11]), "+v"(r[12]), "+v"(r[13]), "+v"(r[14]), "+v"(r[15]))
#define C8 asm volatile("v_cvt_pk_bf16_f32 %0, %0, %1\nv_cvt_pk_bf16_f32 %1, %1, %2\nv_cvt_pk_bf16_f32 %2, %2, %3\nv_cvt_pk_bf16_f32 %3, %3, %4\nv_cvt_pk_bf16_f32 %4, %4, %5\nv_cvt_pk_bf16_f32 %5, %5, %6\nv_cvt_pk_bf16_f32 %6, %6, %7\nv_cvt_pk_bf16_f32 %7, %7, %0\n" : "+v"(c[0]), "+v"(c[1]), "+v"(c[2]), "+v"(c[3]), "+v"(c[4]), "+v"(c[5]), "+v"(c[6]), "+v"(c[7]))

template <int NM, int NE, int NC, int NA = 4, bool AG = false>
__global__ void kern(float* out, int iters) {
  float r[16], c[8];
  for (int i = 0; i < 16; ++i) r[i] = -1.0f / (threadIdx.x + i + 1);
  for (int i = 0; i < 8; ++i) c[i] = 0.5f / (threadIdx.x + i + 1);
  f32x16 acc[4];
  for (int j = 0; j < 4; ++j)
    for (int i = 0; i < 16; ++i) acc[j][i] = 0.f;
  bf16x8 a, b;
  for (int i = 0; i < 8; ++i) a[i] = (__bf16)(threadIdx.x * 0.001f), b[i] = (__bf16)(i * 0.01f);
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < NM; ++j) {
      if constexpr (AG)  // accumulator in AGPRs (separate from the VALU's VGPR operands)
        asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc[j % NA]) : "v"(a), "v"(b));
      else
        acc[j % NA] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[j % NA], 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < NE / 16; ++j) E16;
#pragma unroll
    for (int j = 0; j < NC / 8; ++j) C8;
  }
  float s = 0.f;
  for (int i = 0; i < 16; ++i) s += r[i] + acc[0][i] + acc[1][i] + acc[2][i] + acc[3][i];
  for (int i = 0; i < 8; ++i) s += c[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int NM, int NE, int NC, int NA = 4, bool AG = false>
void run() {
  const int shapes[][2] = {{512, 256}, {512, 512}};
  for (auto& sh : shapes) {
    const int blocks = sh[0], threads = sh[1], iters = 4000;
    float* out;
    (void)hipMalloc(&out, blocks * threads * 4);
    kern<NM, NE, NC, NA, AG><<<blocks, threads>>>(out, iters);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0), (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    kern<NM, NE, NC, NA, AG><<<blocks, threads>>>(out, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double wps = (double)blocks * threads / 64 / 1024;
    const double per = ms * 1e-3 / (iters * wps) * 2.0e9;
    printf("%s chains %d mfma32 x%d + exp x%2d + cvt x%2d  grid %4dx%3d waves/SIMD %.0f: %6.1f cyc/body/SIMD\n", AG ? "agpr" : "vgpr", NA, NM, NE, NC, blocks,
           threads, wps, per);
    (void)hipFree(out);
  }
}

int main() {
  run<4, 0, 0, 4, false>();
  run<4, 0, 0, 4, true>();
  run<4, 16, 8, 4, false>();
  run<4, 16, 8, 4, true>();
  run<4, 16, 0, 4, false>();
  run<4, 16, 0, 4, true>();
  run<4, 32, 16, 4, false>();
  run<4, 32, 16, 4, true>();
  return 0;
}
