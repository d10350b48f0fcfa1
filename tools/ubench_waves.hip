// Microbenchmark (diagnostic tool): does a third wave per SIMD raise the issue-port use of the sample-axis
// attention's step mix?  Each wave runs NCH 32-query chains of the in-wave pipeline the real kernel uses
// (attention_pipe.hip): per 64-key tile and chain 4 score MFMAs (32x32x16) into S(t+1), 32 exps of S(t)
// packed by 16 cvt_pk into P(t), 4 P.V MFMAs and 4 row-sum MFMAs (16x16x32) on P(t) -- the exps depend on the
// previous tile's score MFMAs and the P.V on this tile's conversions, as in the kernel; no memory.
// Launched with W waves per SIMD (blocks of 4 waves; dynamic LDS of 160 KB / W per block caps the CU at W blocks);
// reported: SIMD cycles per
// 64x64 tile-chain pair of work (= the real kernel's per-SIMD step is 2 of these), at the measured wall time.
// Build: hipcc -O3 --offload-arch=gfx950 -mllvm -amdgpu-mfma-vgpr-form=1 tools/ubench_waves.hip -o tools/ubench_waves
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef __attribute__((__vector_size__(16 * sizeof(float)))) float f32x16;
typedef __attribute__((__vector_size__(4 * sizeof(float)))) float f32x4;
typedef __attribute__((__vector_size__(8 * sizeof(__bf16)))) __bf16 bf16x8;

template <int NCH, int W>
__global__ __launch_bounds__(256, W) void kern(float* out, int iters) {
  extern __shared__ float dyn[];  // occupancy cap only
  const int lane = threadIdx.x & 63;
  if (iters < 0) dyn[threadIdx.x] = 0.f;
  bf16x8 q[NCH][2], k[2][2], v[2][2], sel;
  for (int c = 0; c < NCH; ++c)
    for (int i = 0; i < 2; ++i)
      for (int j = 0; j < 8; ++j) q[c][i][j] = (__bf16)(0.001f * (lane + j + c));
  for (int u = 0; u < 2; ++u)
    for (int i = 0; i < 2; ++i)
      for (int j = 0; j < 8; ++j) k[u][i][j] = (__bf16)(0.002f * (lane - j + i)), v[u][i][j] = (__bf16)(0.003f * (j + u));
  for (int j = 0; j < 8; ++j) sel[j] = (__bf16)((lane & 15) == 0 ? 1.f : 0.f);
  f32x16 s[NCH][2], o[NCH];
  f32x4 l[NCH];
  for (int c = 0; c < NCH; ++c) {
    for (int i = 0; i < 16; ++i) s[c][0][i] = s[c][1][i] = o[c][i] = 0.f;
    l[c] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      // exps of S(t) -> P(t) (bf16 fragments)
      bf16x8 p[2][2];
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int sp = 0; sp < 2; ++sp)
#pragma unroll
          for (int j = 0; j < 8; ++j) p[u][sp][j] = (__bf16)__builtin_amdgcn_exp2f(s[c][u][8 * sp + j] * -0.01f);
      // S(t+1) = K Q^T (independent of the exps: the overlap the kernel's pipeline exposes)
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        f32x16 z;
        for (int i = 0; i < 16; ++i) z[i] = 0.f;
        z = __builtin_amdgcn_mfma_f32_32x32x16_bf16(k[u][0], q[c][0], z, 0, 0, 0);
        s[c][u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(k[u][1], q[c][1], z, 0, 0, 0);
      }
      // P.V and row sums on P(t)
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int sp = 0; sp < 2; ++sp) {
          o[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(v[u][sp], p[u][sp], o[c], 0, 0, 0);
          l[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sel, p[u][sp], l[c], 0, 0, 0);
        }
    }
  }
  float acc = 0.f;
  for (int c = 0; c < NCH; ++c)
    for (int i = 0; i < 16; ++i) acc += o[c][i] + s[c][0][i] + s[c][1][i] + (i < 4 ? l[c][i] : 0.f);
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int NCH, int W>
void run(const char* name) {
  const int blocks = 256 * W * 4, threads = 256, iters = 400;
  float* out;
  (void)hipMalloc(&out, (size_t)blocks * threads * 4);
  const size_t lds = (size_t)160 * 1024 / W - 1024;  // at most W blocks (W waves per SIMD) per CU
  (void)hipFuncSetAttribute((const void*)kern<NCH, W>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  kern<NCH, W><<<blocks, threads, lds>>>(out, iters);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0), (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  kern<NCH, W><<<blocks, threads, lds>>>(out, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  // per SIMD: blocks * 4 waves / 1024 SIMDs waves, each iters * NCH tile-chains
  const double chains = (double)blocks * 4 / 1024 * iters * NCH;
  const double cyc = ms * 1e-3 * 2.2e9 / chains;
  printf("%-44s %7.1f SIMD cycles per 64x32 tile-chain (2.2 GHz basis)\n", name, cyc);
  (void)hipFree(out);
}

int main() {
  run<2, 1>("2 chains per wave, 1 wave per SIMD");
  run<2, 2>("2 chains per wave, 2 waves per SIMD (today)");
  run<1, 2>("1 chain per wave, 2 waves per SIMD");
  run<1, 3>("1 chain per wave, 3 waves per SIMD");
  run<1, 4>("1 chain per wave, 4 waves per SIMD");
  run<2, 3>("2 chains per wave, 3 waves per SIMD");
  run<3, 1>("3 chains per wave, 1 wave per SIMD");
  run<4, 1>("4 chains per wave, 1 wave per SIMD");
  return 0;
}
