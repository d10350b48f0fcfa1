// Microbenchmark (diagnostic tool): the sample-axis attention inner loop in isolation, per
// 64-key tile and wave: 8 ds_read_b128 (K, V^T fragments), 8 score MFMAs (two 32-query chains
// x two 32-key halves x K=32), exp2 (optional) + bf16 pack, 8 P.V MFMAs.  Cycles per tile
// per SIMD at 2.0 GHz basis; the MFMA-only bound is 16 x 32 = 512 cycles per tile-wave.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef __attribute__((__vector_size__(16 * sizeof(float)))) float f32x16;
typedef __attribute__((__vector_size__(8 * sizeof(__bf16)))) __bf16 bf16x8;

template <int LDSR, int EXP>
__global__ __launch_bounds__(256, 2) void kern(float* out, int iters) {
  __shared__ __attribute__((aligned(16))) unsigned char lds[8192];
  const int lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < 2048; i += 256) ((float*)lds)[i] = 0.001f * (i % 97);
  __syncthreads();
  bf16x8 qf[2][2], kc[2][2], vc[2][2];
  for (int a = 0; a < 2; ++a)
    for (int b = 0; b < 2; ++b)
      for (int j = 0; j < 8; ++j) {
        qf[a][b][j] = (__bf16)(0.01f * (lane + j + a));
        kc[a][b][j] = (__bf16)(0.02f * (lane - j + b));
        vc[a][b][j] = (__bf16)(0.03f * (j + a + b));
      }
  f32x16 o[2], negm[2];
  for (int a = 0; a < 2; ++a)
    for (int i = 0; i < 16; ++i) o[a][i] = 0.f, negm[a][i] = -1.f;
  bf16x8 kn[2][2], vn[2][2];  // LDSR == 2: next tile's fragments read one iteration ahead
  if (LDSR == 2) {
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        kn[u][i] = *(const bf16x8*)(lds + ((lane & 31) * 64 + 16 * (2 * i + (lane >> 5)) + u * 2048) % 8192);
        vn[u][i] = *(const bf16x8*)(lds + 4096 + ((lane & 31) * 128 + 16 * (2 * (2 * u + i) + (lane >> 5))) % 4096);
      }
  }
  for (int it = 0; it < iters; ++it) {
    negm[0][0] = negm[1][0] = -1.0f - (float)it * 1e-9f;  // loop-variant: the score MFMAs stay in the loop
    bf16x8 kf[2][2], vf[2][2];
    if (LDSR == 2) {
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int i = 0; i < 2; ++i) kf[u][i] = kn[u][i], vf[u][i] = vn[u][i];
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int sh = (it & 1) * 512;  // a different address each iteration
          kn[u][i] = *(const bf16x8*)(lds + ((lane & 31) * 64 + 16 * (2 * i + (lane >> 5)) + u * 2048 + sh) % 8192);
          vn[u][i] = *(const bf16x8*)(lds + 4096 + ((lane & 31) * 128 + 16 * (2 * (2 * u + i) + (lane >> 5)) + sh) % 4096);
        }
      __builtin_amdgcn_sched_barrier(0);  // the next tile's reads stay ahead of this tile's MFMAs
    } else if (LDSR) {
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          kf[u][i] = *(const bf16x8*)(lds + ((lane & 31) * 64 + 16 * (2 * i + (lane >> 5)) + u * 2048) % 8192);
          vf[u][i] = *(const bf16x8*)(lds + 4096 + ((lane & 31) * 128 + 16 * (2 * (2 * u + i) + (lane >> 5))) % 4096);
        }
    } else {
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int i = 0; i < 2; ++i) kf[u][i] = kc[u][i], vf[u][i] = vc[u][i];
    }
    f32x16 s[2][2];
#pragma unroll
    for (int qb = 0; qb < 2; ++qb)
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        s[qb][u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[u][0], qf[qb][0], negm[qb], 0, 0, 0);
        s[qb][u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[u][1], qf[qb][1], s[qb][u], 0, 0, 0);
      }
#pragma unroll
    for (int qb = 0; qb < 2; ++qb)
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int sp = 0; sp < 2; ++sp) {
          bf16x8 pb;
#pragma unroll
          for (int j = 0; j < 8; ++j)
            pb[j] = (__bf16)(EXP ? __builtin_amdgcn_exp2f(s[qb][u][8 * sp + j]) : s[qb][u][8 * sp + j]);
          o[qb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf[u][sp], pb, o[qb], 0, 0, 0);
        }
  }
  float r = 0.f;
  for (int i = 0; i < 16; ++i) r += o[0][i] + o[1][i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <int LDSR, int EXP>
void run(const char* name) {
  for (int blocks : {256, 512}) {
    const int iters = 2000;
    float* out;
    (void)hipMalloc(&out, blocks * 256 * 4);
    kern<LDSR, EXP><<<blocks, 256>>>(out, iters);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0), (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    kern<LDSR, EXP><<<blocks, 256>>>(out, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double wps = (double)blocks * 4 / 1024;
    const double per = ms * 1e-3 / (iters * wps) * 2.0e9;
    printf("%-22s waves/SIMD %.0f: %6.1f cyc per tile-wave (MFMA bound 512)\n", name, wps, per);
    (void)hipFree(out);
  }
}

int main() {
  run<0, 0>("regs, no exp");
  run<1, 0>("lds, no exp");
  run<2, 0>("lds ahead, no exp");
  run<0, 1>("regs, exp");
  run<1, 1>("lds, exp");
  return 0;
}
