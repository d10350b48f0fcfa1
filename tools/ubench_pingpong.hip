// Microbenchmark (diagnostic tool): two waves per SIMD (512-thread block, waves w and w+4 share a
// SIMD), wave group 0 issuing only v_mfma_f32_32x32x16_bf16 and group 1 only v_exp_f32 (+ cvt_pk),
// alone and together: do the matrix pipe and the transcendental issue of two partner waves overlap?
// cycles per iteration per SIMD at the measured wall time (2.0 GHz basis).
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef __attribute__((__vector_size__(16 * sizeof(float)))) float f32x16;
typedef __attribute__((__vector_size__(8 * sizeof(__bf16)))) __bf16 bf16x8;

#define E16 asm volatile("v_exp_f32 %0, %0\nv_exp_f32 %1, %1\nv_exp_f32 %2, %2\nv_exp_f32 %3, %3\nv_exp_f32 %4, %4\nv_exp_f32 %5, %5\nv_exp_f32 %6, %6\nv_exp_f32 %7, %7\nv_exp_f32 %8, %8\nv_exp_f32 %9, %9\nv_exp_f32 %10, %10\nv_exp_f32 %11, %11\nv_exp_f32 %12, %12\nv_exp_f32 %13, %13\nv_exp_f32 %14, %14\nv_exp_f32 %15, %15\n" : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7]), "+v"(r[8]), "+v"(r[9]), "+v"(r[10]), "+v"(r[11]), "+v"(r[12]), "+v"(r[13]), "+v"(r[14]), "+v"(r[15]))
#define C8 asm volatile("v_cvt_pk_bf16_f32 %0, %8, %9\nv_cvt_pk_bf16_f32 %1, %9, %10\nv_cvt_pk_bf16_f32 %2, %10, %11\nv_cvt_pk_bf16_f32 %3, %11, %12\nv_cvt_pk_bf16_f32 %4, %12, %13\nv_cvt_pk_bf16_f32 %5, %13, %14\nv_cvt_pk_bf16_f32 %6, %14, %15\nv_cvt_pk_bf16_f32 %7, %15, %8\n" : "=v"(c[0]), "=v"(c[1]), "=v"(c[2]), "=v"(c[3]), "=v"(c[4]), "=v"(c[5]), "=v"(c[6]), "=v"(c[7]) : "v"(r[0]), "v"(r[1]), "v"(r[2]), "v"(r[3]), "v"(r[4]), "v"(r[5]), "v"(r[6]), "v"(r[7]))

// MODE bit 0: group 0 runs NM MFMAs per iteration; bit 1: group 1 runs NE exps (+ NE/2 cvt);
// MODE 4: every wave runs both (the unsplit schedule)
template <int MODE, int NM, int NE, int PRIO>
__global__ __launch_bounds__(512, 1) void kern(float* out, int iters) {
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int grp = wave >> 2;
  float r[16];
  unsigned c[8];
  for (int i = 0; i < 16; ++i) r[i] = -1.0f / (threadIdx.x + i + 1);
  for (int i = 0; i < 8; ++i) c[i] = 0;
  f32x16 acc[4];
  for (int j = 0; j < 4; ++j)
    for (int i = 0; i < 16; ++i) acc[j][i] = 0.f;
  bf16x8 a, b;
  for (int i = 0; i < 8; ++i) a[i] = (__bf16)(threadIdx.x * 0.001f), b[i] = (__bf16)(i * 0.01f);
  const bool do_m = MODE == 4 || ((MODE & 1) && grp == 0);
  const bool do_e = MODE == 4 || ((MODE & 2) && grp == 1);
  if (PRIO && do_m && MODE != 4) __builtin_amdgcn_s_setprio(1);
  for (int it = 0; it < iters; ++it) {
    if (do_m) {
#pragma unroll
      for (int j = 0; j < NM; ++j) acc[j & 3] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[j & 3], 0, 0, 0);
    }
    if (do_e) {
#pragma unroll
      for (int j = 0; j < NE / 16; ++j) {
        E16;
        C8;
      }
    }
  }
  float s = 0.f;
  for (int i = 0; i < 16; ++i) s += r[i] + acc[0][i] + acc[1][i] + acc[2][i] + acc[3][i];
  for (int i = 0; i < 8; ++i) s += (float)c[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int MODE, int NM, int NE, int PRIO = 0>
void run(const char* name) {
  const int blocks = 256 * 4, threads = 512, iters = 2000;
  float* out;
  (void)hipMalloc(&out, blocks * threads * 4);
  kern<MODE, NM, NE, PRIO><<<blocks, threads>>>(out, iters);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0), (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  kern<MODE, NM, NE, PRIO><<<blocks, threads>>>(out, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  // blocks / 256 CUs rounds, each iteration of one block = one iteration per SIMD
  const double per = ms * 1e-3 / (iters * (blocks / 256.0)) * 2.0e9;
  printf("%-40s %7.1f cyc/iter/SIMD\n", name, per);
  (void)hipFree(out);
}

int main() {
  run<1, 16, 64>("G0 16 mfma32 alone");
  run<2, 16, 64>("G1 64 exp + 32 cvt alone");
  run<3, 16, 64>("G0 mfma | G1 exp (split)");
  run<3, 16, 64, 1>("G0 mfma prio1 | G1 exp (split)");
  run<4, 8, 32>("all: 8 mfma + 32 exp each (unsplit)");
  run<1, 16, 0>("G0 16 mfma32 alone (no exp code)");
  run<3, 16, 32>("G0 mfma | G1 32 exp");
  return 0;
}
