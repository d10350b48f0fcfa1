// Row-resident MLP sublayer for gfx950 (bf16 performance mode):
//   X <- LayerNorm(X + GELU(X W1^T) W2^T)           (mlp.py:93-104, layer.py:437-455)
//
// Each wave owns 32 rows for the whole sublayer and keeps them in registers:
//   * its rows of X, as bf16 B-operand fragments (A^T), loaded once from HBM;
//   * the hidden activations of the current 32-wide hidden chunk, computed
//     transposed (H^T = W1c . A^T) so the accumulator of one 16x16 tile pair is,
//     lane for lane, the B operand of the down projection (Y^T += W2c . H^T) once the
//     chunk's K order is permuted (pos 8g+j <-> hidden 4g+j / 16+4g+j-4; W2 is stored
//     in that order, see pack_mlp2_perm in capi.cpp);
//   * the 192 x 32 output accumulator Y^T, then residual + LayerNorm across lanes.
// Only the weights move through LDS: a 128-row block (4 waves) shares each 32-wide
// hidden chunk of W1 (32 x 192) and W2 (192 x 32), double buffered, one barrier per
// chunk, so weight bytes per row are a quarter of a 32-row tiling and X is read once
// and written once.
#include "common.h"
#include "kernels.h"

namespace mmpfn {

namespace {

constexpr int RE = 192;               // model width
constexpr int RHC = 32;               // hidden chunk
constexpr int RROWS = 128;            // rows per block (4 waves x 32)
constexpr int W1ST = RE + 16;         // W1 chunk LDS row stride (bf16): 416 B (32 mod 64: conflict-free b128)
constexpr int W2ST = RHC + 16;        // W2 chunk LDS row stride (bf16): 96 B
constexpr int W1EL = RHC * W1ST;      // 6400
constexpr int BUFEL = W1EL + RE * W2ST;  // 6656 + 9216 bf16 per buffer
constexpr int PIECES = (RHC * RE + RE * RHC) / 8 / 256;  // 16-B pieces per thread per chunk (6)

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__global__ __launch_bounds__(256, 2) void mlp_rows_kernel(float* __restrict__ X, const bf16* __restrict__ W1,
                                                          const bf16* __restrict__ W2p, int M, int Fh, float eps) {
  __shared__ __attribute__((aligned(16))) bf16 wbuf[2 * BUFEL];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const int64_t m0 = (int64_t)blockIdx.x * RROWS + wave * 32;
  const int nchunks = Fh / RHC;

  // chunk c pieces: [0, 768) W1 rows c*32.. (24 pieces of 16 B per row), [768, 1536) W2 rows (4 per row)
  u32x4 pf[PIECES];
  auto fetch = [&](int c) {
#pragma unroll
    for (int j = 0; j < PIECES; ++j) {
      const int p = tid + 256 * j;
      if (j < PIECES / 2) {
        pf[j] = *(const u32x4*)(W1 + (int64_t)(c * RHC + p / 24) * RE + (p % 24) * 8);
      } else {
        const int q = p - RHC * RE / 8;
        pf[j] = *(const u32x4*)(W2p + (int64_t)(q >> 2) * Fh + c * RHC + (q & 3) * 8);
      }
    }
  };
  auto stash = [&](int buf) {
    bf16* b = wbuf + buf * BUFEL;
#pragma unroll
    for (int j = 0; j < PIECES; ++j) {
      const int p = tid + 256 * j;
      if (j < PIECES / 2) {
        *(u32x4*)(b + (p / 24) * W1ST + (p % 24) * 8) = pf[j];
      } else {
        const int q = p - RHC * RE / 8;
        *(u32x4*)(b + W1EL + (q >> 2) * W2ST + (q & 3) * 8) = pf[j];
      }
    }
  };

  fetch(0);
  // the wave's rows as A^T fragments: lane = row (tile tt, col fr), 8 consecutive features
  bf16x8 af[2][RE / 32];
#pragma unroll
  for (int tt = 0; tt < 2; ++tt) {
    const int64_t m = min(m0 + tt * 16 + fr, (int64_t)M - 1);
    const float* xr = X + m * RE + fg * 8;
#pragma unroll
    for (int ks = 0; ks < RE / 32; ++ks) {
      const f32x4 lo = *(const f32x4*)(xr + ks * 32);
      const f32x4 hi = *(const f32x4*)(xr + ks * 32 + 4);
      bf16x8 b;
      b[0] = (bf16)lo[0], b[1] = (bf16)lo[1], b[2] = (bf16)lo[2], b[3] = (bf16)lo[3];
      b[4] = (bf16)hi[0], b[5] = (bf16)hi[1], b[6] = (bf16)hi[2], b[7] = (bf16)hi[3];
      af[tt][ks] = b;
    }
  }
  stash(0);
  __syncthreads();

  f32x4 y[RE / 16][2];
#pragma unroll
  for (int o = 0; o < RE / 16; ++o) y[o][0] = y[o][1] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int c = 0; c < nchunks; ++c) {
    if (c + 1 < nchunks) fetch(c + 1);
    const bf16* w1 = wbuf + (c & 1) * BUFEL;
    const bf16* w2 = w1 + W1EL;
    // H^T [32 hidden][32 rows] = W1c . A^T
    f32x4 h[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i) h[i][0] = h[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
    // W1 fragments one k-step ahead of the MFMAs (sched barriers keep the reads early)
    bf16x8 wa[2][2];
#pragma unroll
    for (int ht = 0; ht < 2; ++ht) wa[0][ht] = *(const bf16x8*)(w1 + (ht * 16 + fr) * W1ST + fg * 8);
#pragma unroll
    for (int ks = 0; ks < RE / 32; ++ks) {
      if (ks + 1 < RE / 32) {
#pragma unroll
        for (int ht = 0; ht < 2; ++ht)
          wa[(ks + 1) & 1][ht] = *(const bf16x8*)(w1 + (ht * 16 + fr) * W1ST + (ks + 1) * 32 + fg * 8);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int ht = 0; ht < 2; ++ht)
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) h[ht][tt] = mfma16(wa[ks & 1][ht], af[tt][ks], h[ht][tt]);
    }
    // GELU; the two hidden tiles' rows 4g..4g+3 form this lane's permuted K=32 B fragment
    bf16x8 hb[2];
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        hb[tt][i] = (bf16)gelu_tanh_fast(h[0][tt][i]);
        hb[tt][4 + i] = (bf16)gelu_tanh_fast(h[1][tt][i]);
      }
    }
    // Y^T [192][32 rows] += W2c(perm) . H^T
    // W2 fragments in groups of 4 output tiles, the next group's reads issued first
    bf16x8 wb[2][4];
#pragma unroll
    for (int i = 0; i < 4; ++i) wb[0][i] = *(const bf16x8*)(w2 + (i * 16 + fr) * W2ST + fg * 8);
#pragma unroll
    for (int og = 0; og < RE / 64; ++og) {
      if (og + 1 < RE / 64) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          wb[(og + 1) & 1][i] = *(const bf16x8*)(w2 + (((og + 1) * 4 + i) * 16 + fr) * W2ST + fg * 8);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) y[og * 4 + i][tt] = mfma16(wb[og & 1][i], hb[tt], y[og * 4 + i][tt]);
    }
    if (c + 1 < nchunks) stash((c + 1) & 1);
    __syncthreads();
  }

  // residual + LayerNorm: lane = row, 48 of its 192 features (rows 16o + 4g + i of Y^T)
#pragma unroll
  for (int tt = 0; tt < 2; ++tt) {
    const int64_t m = m0 + tt * 16 + fr;
    const bool valid = m < M;
    float* xr = X + (valid ? m : (int64_t)M - 1) * RE + fg * 4;
    float s = 0.f;
#pragma unroll
    for (int o = 0; o < RE / 16; ++o) {
      const f32x4 xv = *(const f32x4*)(xr + o * 16);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        y[o][tt][i] += xv[i];
        s += y[o][tt][i];
      }
    }
    s = sum_rows4(s);
    const float mean = s * (1.0f / RE);
    float q = 0.f;
#pragma unroll
    for (int o = 0; o < RE / 16; ++o)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float dl = y[o][tt][i] - mean;
        q += dl * dl;
      }
    q = sum_rows4(q);
    const float inv = 1.0f / sqrtf(q * (1.0f / RE) + eps);
    if (valid) {
#pragma unroll
      for (int o = 0; o < RE / 16; ++o) {
        f32x4 ov;
#pragma unroll
        for (int i = 0; i < 4; ++i) ov[i] = (y[o][tt][i] - mean) * inv;
        *(f32x4*)(xr + o * 16) = ov;
      }
    }
  }
}

}  // namespace

hipError_t launch_mlp_rows(float* X, const void* W1, const void* W2perm, int64_t M, int E, int Fh, float eps,
                           hipStream_t st) {
  if (M <= 0) return hipSuccess;
  if (E != RE || Fh % RHC != 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(mlp_rows_kernel, dim3((unsigned)((M + RROWS - 1) / RROWS)), dim3(256), 0, st, X,
                     (const bf16*)W1, (const bf16*)W2perm, (int)M, Fh, eps);
  return hipGetLastError();
}

}  // namespace mmpfn
