// Microbenchmark (diagnostic tool): the MLP chunk's instruction mix (mlp_rows.hip) without memory -- does the
// 32x32x16 MFMA form (half the MFMA issue holds of 16x16x32 for the same flops) run a chunk faster at two waves per
// SIMD?  Per chunk and wave: the up-projection (32 hidden x 32 rows x 192) and the down-projection (192 x 32 rows x
// 32 hidden) = 48 v_mfma_f32_16x16x32_f16 or 24 v_mfma_f32_32x32x16_f16, the previous chunk's GELU on 16 values
// per lane in packed fp16 (gelu_tanh_h2: 2 transcendentals per value), and 24 ds_read_b128 of weight fragments.
// Build: hipcc -O3 --offload-arch=gfx950 -mllvm -amdgpu-mfma-vgpr-form=1 tools/ubench_mlp.hip -o tools/ubench_mlp
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef __attribute__((__vector_size__(16 * sizeof(float)))) float f32x16;
typedef __attribute__((__vector_size__(4 * sizeof(float)))) float f32x4;
typedef __attribute__((__vector_size__(8 * sizeof(_Float16)))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(2))) _Float16 f16x2_t;

__device__ __forceinline__ f16x2_t gelu_h2(f16x2_t x) {
  constexpr float k = -2.0f * 0.7978845608028654f * 1.4426950408889634f;
  const f16x2_t kk = {(_Float16)k, (_Float16)k}, kc = {(_Float16)(k * 0.044715f), (_Float16)(k * 0.044715f)};
  const f16x2_t one = {(_Float16)1.0f, (_Float16)1.0f};
  const f16x2_t u = x * __builtin_elementwise_fma(kc, x * x, kk);
  const f16x2_t d = f16x2_t{(_Float16)__builtin_exp2f16(u[0]), (_Float16)__builtin_exp2f16(u[1])} + one;
  return x * f16x2_t{(_Float16)__builtin_amdgcn_rcph(d[0]), (_Float16)__builtin_amdgcn_rcph(d[1])};
}

template <bool BIG, bool GELU, bool LDS>
__global__ __launch_bounds__(256, 2) void kern(float* out, int iters) {
  __shared__ f16x8 w[64 * 24];
  const int lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < 64 * 24; i += 256)
    for (int j = 0; j < 8; ++j) w[i][j] = (_Float16)(0.001f * (i + j));
  __syncthreads();
  f16x8 a[6], wf[4];
  for (int k = 0; k < 6; ++k)
    for (int j = 0; j < 8; ++j) a[k][j] = (_Float16)(0.01f * (lane + k - j));
  for (int k = 0; k < 4; ++k)
    for (int j = 0; j < 8; ++j) wf[k][j] = (_Float16)(0.02f * (k + j));
  f32x4 y16[12][2], h16[2][2];
  f32x16 y32[6], h32;
  for (int i = 0; i < 12; ++i) y16[i][0] = y16[i][1] = f32x4{0, 0, 0, 0};
  for (int i = 0; i < 6; ++i) y32[i] = f32x16{};
  h16[0][0] = h16[0][1] = h16[1][0] = h16[1][1] = f32x4{0.1f, 0.2f, 0.3f, 0.4f};
  h32 = f32x16{};
  f16x8 hb[2];
  for (int j = 0; j < 8; ++j) hb[0][j] = (_Float16)(0.1f * j), hb[1][j] = (_Float16)(0.2f * j + 0.05f);
  for (int it = 0; it < iters; ++it) {
    // GELU of the previous chunk (16 values per lane) -> the down-projection's B fragments
    if constexpr (GELU) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          f16x2_t v = {(_Float16)(BIG ? h32[8 * t + 2 * q] : h16[t][q >> 1][2 * (q & 1)]),
                       (_Float16)(BIG ? h32[8 * t + 2 * q + 1] : h16[t][q >> 1][2 * (q & 1) + 1])};
          v = gelu_h2(v);
          hb[t][2 * q] = v[0], hb[t][2 * q + 1] = v[1];
        }
    }
    // up-projection of the next chunk
    if constexpr (BIG) {
      f32x16 h = {};
#pragma unroll
      for (int k = 0; k < 12; ++k) {
        if (LDS && (k & 1) == 0) wf[k & 3] = w[(lane + 64 * k) % (64 * 24)];
        h = __builtin_amdgcn_mfma_f32_32x32x16_f16(wf[k & 3], a[k % 6], h, 0, 0, 0);
      }
      h32 = h;
    } else {
      f32x4 h[2][2] = {};
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        if (LDS) wf[k & 3] = w[(lane + 64 * k) % (64 * 24)], wf[(k + 1) & 3] = w[(lane + 64 * k + 32) % (64 * 24)];
#pragma unroll
        for (int ht = 0; ht < 2; ++ht)
#pragma unroll
          for (int tt = 0; tt < 2; ++tt) h[ht][tt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[(k + ht) & 3], a[(k + 3 * tt) % 6], h[ht][tt], 0, 0, 0);
      }
      for (int i = 0; i < 2; ++i) h16[i][0] = h[i][0], h16[i][1] = h[i][1];
    }
    // down-projection of this chunk
    if constexpr (BIG) {
#pragma unroll
      for (int o = 0; o < 6; ++o) {
        if (LDS) wf[o & 3] = w[(lane + 64 * (o + 12)) % (64 * 24)];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) y32[o] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wf[o & 3], hb[ks], y32[o], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int o = 0; o < 12; ++o) {
        if (LDS) wf[o & 3] = w[(lane + 64 * (o + 12)) % (64 * 24)];
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) y16[o][tt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[o & 3], hb[tt], y16[o][tt], 0, 0, 0);
      }
    }
  }
  float s = 0.f;
  for (int i = 0; i < 12; ++i) s += y16[i][0][0] + y16[i][1][1];
  for (int i = 0; i < 6; ++i) s += y32[i][0] + y32[i][5];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s + h32[3] + h16[0][0][1];
}

template <bool BIG, bool GELU, bool LDS>
void run(const char* name) {
  const int blocks = 256 * 2 * 4, threads = 256, iters = 300;
  float* out;
  (void)hipMalloc(&out, (size_t)blocks * threads * 4);
  kern<BIG, GELU, LDS><<<blocks, threads>>>(out, iters);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0), (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  kern<BIG, GELU, LDS><<<blocks, threads>>>(out, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double chunks = (double)blocks * 4 / 1024 * iters;  // per SIMD
  printf("%-52s %7.1f SIMD cycles per chunk-wave (2.2 GHz basis)\n", name, ms * 1e-3 * 2.2e9 / chunks);
  (void)hipFree(out);
}

int main() {
  run<false, false, false>("16x16x32: MFMAs only");
  run<true, false, false>("32x32x16: MFMAs only");
  run<false, true, false>("16x16x32: MFMAs + GELU");
  run<true, true, false>("32x32x16: MFMAs + GELU");
  run<false, true, true>("16x16x32: MFMAs + GELU + LDS fragment reads");
  run<true, true, true>("32x32x16: MFMAs + GELU + LDS fragment reads");
  return 0;
}
