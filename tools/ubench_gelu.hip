// Microbenchmark (diagnostic tool): the MLP chunk's GELU forms in the chunk's MFMA mix (mlp_rows.hip, fp16 mode)
// without memory.  Per chunk and wave: 48 v_mfma_f32_16x16x32_f16 (up- and down-projection of 32 hidden x 32 rows
// x 192 features) and the previous chunk's GELU on 16 fp32 accumulator values per lane, packed into fp16 B fragments.
// GELU forms: 0 none; 1 tanh form in packed fp16 (gelu_tanh_h2, today's); 2 tanh form in fp32 (gelu_tanh_fast);
// 3 exact-erf GELU as x * (1/2 + t P(t^2)), t = clamp(x / 4.5, -1, 1), P of degree 8 in packed fp32
// (v_pk_fma_f32), no transcendental; 4 form 3 with the clamp folded into one v_med3 per element.
// Build: hipcc -O3 --offload-arch=gfx950 -mllvm -amdgpu-mfma-vgpr-form=1 tools/ubench_gelu.hip -o tools/ubench_gelu
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "../multimodalpfn_amd/csrc/common.h"
using namespace mmpfn;
typedef __attribute__((ext_vector_type(2))) float f2;

__device__ __forceinline__ f2 gelu_poly2(f2 x) {
  const f2 t = {__builtin_amdgcn_fmed3f(x[0] * (1.f / 4.5f), -1.f, 1.f), __builtin_amdgcn_fmed3f(x[1] * (1.f / 4.5f), -1.f, 1.f)};
  const f2 t2 = t * t;
  f2 q = {4.605697077e+00f, 4.605697077e+00f};
  const float c[8] = {-2.414337839e+01f, 5.552828972e+01f, -7.436876462e+01f, 6.518081225e+01f,
                      -3.997702372e+01f, 1.791278917e+01f, -6.033250355e+00f, 1.794838832e+00f};
#pragma unroll
  for (int k = 0; k < 8; ++k) q = __builtin_elementwise_fma(q, t2, f2{c[k], c[k]});
  return x * __builtin_elementwise_fma(t, q, f2{0.5f, 0.5f});
}

template <int G>
__device__ __forceinline__ f16x2_t gelu2(float a, float b) {
  if constexpr (G == 1) return gelu_tanh_h2(f16x2_t{(_Float16)a, (_Float16)b});
  else if constexpr (G == 2) return f16x2_t{(_Float16)gelu_tanh_fast(a), (_Float16)gelu_tanh_fast(b)};
  else {
    const f2 g = gelu_poly2(f2{a, b});
    return f16x2_t{(_Float16)g[0], (_Float16)g[1]};
  }
}

template <int G, bool MF>
__global__ __launch_bounds__(256, 2) void kern(float* out, int iters) {
  const int lane = threadIdx.x & 63;
  f16x8 a[6], wf[4];
  for (int k = 0; k < 6; ++k)
    for (int j = 0; j < 8; ++j) a[k][j] = (_Float16)(0.01f * (lane + k - j));
  for (int k = 0; k < 4; ++k)
    for (int j = 0; j < 8; ++j) wf[k][j] = (_Float16)(0.02f * (k + j) - 0.05f);
  f32x4 y16[12][2], h16[2][2];
  for (int i = 0; i < 12; ++i) y16[i][0] = y16[i][1] = f32x4{0, 0, 0, 0};
  for (int i = 0; i < 2; ++i) h16[i][0] = h16[i][1] = f32x4{0.1f * lane, -0.2f, 0.3f, -0.4f * i};
  f16x8 hb[2];
  for (int j = 0; j < 8; ++j) hb[0][j] = (_Float16)(0.1f * j), hb[1][j] = (_Float16)(0.2f * j + 0.05f);
  for (int it = 0; it < iters; ++it) {
    if constexpr (G != 0) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f16x2_t v = gelu2<G>(h16[t][q >> 1][2 * (q & 1)], h16[t][q >> 1][2 * (q & 1) + 1]);
          hb[t][2 * q] = v[0], hb[t][2 * q + 1] = v[1];
        }
    }
    if constexpr (MF) {
      f32x4 h[2][2] = {};
#pragma unroll
      for (int k = 0; k < 6; ++k)
#pragma unroll
        for (int ht = 0; ht < 2; ++ht)
#pragma unroll
          for (int tt = 0; tt < 2; ++tt)
            h[ht][tt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[(k + ht) & 3], a[(k + 3 * tt) % 6], h[ht][tt], 0, 0, 0);
      for (int i = 0; i < 2; ++i) h16[i][0] = h[i][0], h16[i][1] = h[i][1];
#pragma unroll
      for (int o = 0; o < 12; ++o)
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) y16[o][tt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[o & 3], hb[tt], y16[o][tt], 0, 0, 0);
    } else {  // GELU alone: feed the result back so the chain stays live
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) h16[i][j][e] = 0.5f * (float)hb[i][4 * j + e] - 0.25f * h16[i][j][e];
    }
  }
  float s = 0.f;
  for (int i = 0; i < 12; ++i) s += y16[i][0][0] + y16[i][1][1];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s + h16[0][0][1] + h16[1][1][2] + (float)hb[1][3];
}

template <int G, bool MF>
void run(const char* name) {
  const int blocks = 256 * 2 * 4, threads = 256, iters = 300;
  float* out;
  (void)hipMalloc(&out, (size_t)blocks * threads * 4);
  kern<G, MF><<<blocks, threads>>>(out, iters);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0), (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  kern<G, MF><<<blocks, threads>>>(out, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double chunks = (double)blocks * 4 / 1024 * iters;  // chunk-waves per SIMD
  printf("%-50s %7.1f SIMD cycles per chunk-wave (2.2 GHz basis)\n", name, ms * 1e-3 * 2.2e9 / chunks);
  (void)hipFree(out);
}

int main() {
  run<1, false>("GELU alone: tanh form, packed fp16 (today)");
  run<2, false>("GELU alone: tanh form, fp32");
  run<3, false>("GELU alone: erf polynomial, packed fp32");
  run<0, true>("MFMAs, no GELU");
  run<1, true>("MFMAs + tanh form, packed fp16 (today)");
  run<2, true>("MFMAs + tanh form, fp32");
  run<3, true>("MFMAs + erf polynomial, packed fp32");
  run<1, true>("MFMAs + tanh form, packed fp16 (today, again)");
  run<3, true>("MFMAs + erf polynomial, packed fp32 (again)");
  return 0;
}
