// Microbenchmark (diagnostic tool, not product code): per-SIMD issue throughput of the
// softmax instruction mix on gfx950.  Each wave runs ITER iterations of a body; cycles per
// body from s_memtime, averaged over waves; waves/SIMD set by the block size.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) float f32x4;

template <int MODE>
__global__ void kern(float* out, unsigned long long* cyc, int iters) {
  float v[16];
  for (int i = 0; i < 16; ++i) v[i] = (threadIdx.x + i) * 1e-3f - 0.5f;
  f32x16 acc = {}, acc2 = {};
  f32x4 acc3 = {};
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) a[j] = (__bf16)(threadIdx.x * 1e-3f), b[j] = (__bf16)(j * 1e-2f);
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    if (MODE == 0 || MODE == 2 || MODE == 3) {  // 16 exps
#pragma unroll
      for (int i = 0; i < 16; ++i) v[i] = __builtin_amdgcn_exp2f(v[i]) - 1.0f * (MODE == 3 ? 0.f : 0.f);
    }
    if (MODE == 1) {  // 16 fma
#pragma unroll
      for (int i = 0; i < 16; ++i) v[i] = fmaf(v[i], 0.999f, 1e-3f);
    }
    if (MODE == 2 || MODE == 4) {  // 2 MFMA 32x32x16 (64 cycles of matrix pipe)
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
    }
    if (MODE == 6 || MODE == 7) {  // attention mix: 16 exp + 8 cvt_pk + 4 mfma32 + 2 mfma16
#pragma unroll
      for (int i = 0; i < 16; ++i) v[i] = __builtin_amdgcn_exp2f(v[i]);
      bf16x8 pb;
#pragma unroll
      for (int i = 0; i < 8; ++i) pb[i] = (__bf16)(v[i] + v[i + 8]);
      if (MODE == 6) {
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
        acc2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, pb, acc2, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b, a, acc, 0, 0, 0);
        acc2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pb, a, acc2, 0, 0, 0);
        acc3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, pb, acc3, 0, 0, 0);
        acc3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b, pb, acc3, 0, 0, 0);
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) v[i] = v[i] * 1e-30f + (float)pb[i & 7];
    }
    if (MODE == 8) {  // mfma only: 4 mfma32 + 2 mfma16, independent chains
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
        acc2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc2, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b, a, acc, 0, 0, 0);
        acc2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b, a, acc2, 0, 0, 0);
        acc3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc3, 0, 0, 0);
        acc3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b, b, acc3, 0, 0, 0);
    }
    if (MODE == 5) {  // 16 exp (f16)
#pragma unroll
      for (int i = 0; i < 16; ++i) v[i] = (float)__builtin_amdgcn_exp2f((float)(_Float16)v[i]);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0;
  for (int i = 0; i < 16; ++i) s += v[i] + acc[i] + acc2[i] + acc3[i & 3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <int MODE>
void run(const char* name, int threads, int iters) {
  const int blocks = 256 * 2;
  float* out;
  unsigned long long* cyc;
  hipMalloc(&out, blocks * threads * 4);
  hipMalloc(&cyc, blocks * threads / 64 * 8);
  kern<MODE><<<blocks, threads>>>(out, cyc, iters);
  hipEvent_t e0, e1;
  hipEventCreate(&e0), hipEventCreate(&e1);
  hipEventRecord(e0);
  kern<MODE><<<blocks, threads>>>(out, cyc, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const int nw = blocks * threads / 64;
  unsigned long long* h = new unsigned long long[nw];
  hipMemcpy(h, cyc, nw * 8, hipMemcpyDeviceToHost);
  double avg = 0;
  for (int i = 0; i < nw; ++i) avg += h[i];
  avg /= nw;
  // waves per SIMD = blocks * (threads/64) / 1024 (all resident)
  const double wps = (double)blocks * threads / 64 / 1024;
  printf("%-28s waves/SIMD %.1f: %7.1f cyc per body per wave, %6.1f cyc per body per SIMD, %.3f ms\n", name, wps,
         avg / iters, avg / iters / wps, ms);
  delete[] h;
  hipFree(out), hipFree(cyc);
}

int main() {
  for (int t : {128, 256, 512}) {
    run<0>("16 exp", t, 4000);
    run<6>("attn mix (16e 8c 4M32 2M16)", t, 4000);
    run<7>("attn mix without mfma", t, 4000);
    run<8>("mfma only 4M32 2M16", t, 4000);
  }
  return 0;
}
