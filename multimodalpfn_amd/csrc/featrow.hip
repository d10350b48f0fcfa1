// Row-resident attention-between-features sublayer for gfx950 (bf16 performance mode):
//   X <- LayerNorm(X + MHA_features(X))        (layer.py:332-339,437-455; multi_head_attention.py:547-736)
//
// One wave owns one table row (its T <= 16*NT tokens) for the whole sublayer and never
// moves the row's data through LDS: every MFMA result is, lane for lane, the operand of the
// next MFMA (v_mfma_f32_16x16x32_bf16; lane l = (g = l>>4, n = l&15)):
//   X^T fragments     xf[tt][ks]  lane holds X[token 16tt+n][32ks+8g .. +7]            (B / A operand)
//   Q^T, K^T tiles    = W_{q,k} . X^T, W rows permuted so that tile f row 4g+i is head dim 8g+4f+i:
//                      the two tiles of a token tile concatenate into the lane's Q[token][8g..8g+7]
//                      -- the B operand (Q^T) and the A operand (K) of S^T = K Q^T
//   V tiles           = X . Wv^T (untransposed): lane holds V[token 16kt+4g+i][d = 16mt+n], two key
//                      tiles concatenate into the A operand V^T[d][keys] of O^T = V^T P^T, in the
//                      same permuted key order as P^T taken from the S^T accumulators
//   O^T tiles         lane holds O^T[d 16mt+4g+i][query n]; concatenated over mt they are the B
//                      operand of Y^T += Wout_h . O^T with Wout's 32 head columns permuted alike
//   Y^T accumulators  lane holds Y^T[feature 16f+4g+i][token n]: residual + LayerNorm per token
//                      with the 48 features of a lane reduced across the 4 lane groups.
// The softmax scale log2(e)/sqrt(32) is folded into Wq (exp2 on the scores).
// Only the weights move: per head one 48 KB pack (96 x 192 QKV slice + 192 x 32 Wout slice,
// capi.cpp pack_feat_rows) is staged in LDS for the block's 4 waves (4 rows), double
// buffered, the next head's pack in flight during the current head.
// Per row and head: 18*NT MFMAs for QKV, NT^2 for S^T, 2*NT*ceil(NT/2) for P.V, 12*NT for the
// out-projection; HBM traffic = X read + X written once.
#include "common.h"
#include "kernels.h"

namespace mmpfn {

namespace {

constexpr int FR_E = 192;                     // model width
constexpr int FR_H = 6;                       // heads
constexpr int FR_QKV_ST = FR_E + 16;          // LDS row stride (bf16) of the 96 x 192 QKV slice: 416 B
constexpr int FR_OUT_ST = 48;                 // LDS row stride (bf16) of the 192 x 32 Wout slice: 96 B
constexpr int FR_QKV_EL = 96 * FR_QKV_ST;     // 19968
constexpr int FR_BUF_EL = FR_QKV_EL + FR_E * FR_OUT_ST;  // 29184 bf16 per buffer
constexpr int FR_PIECES = FEAT_PACK_HEAD / 8 / 256;       // 16-B pieces per thread and head (12)
constexpr int FR_QKV_PIECES = 96 * FR_E / 8 / 256;        // of which QKV (9)

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ bf16x8 cat8(const f32x4& a, const f32x4& b, float s = 1.0f) {
  bf16x8 r;
#pragma unroll
  for (int i = 0; i < 4; ++i) r[i] = (bf16)(a[i] * s), r[4 + i] = (bf16)(b[i] * s);
  return r;
}

template <int NT>
__global__ __launch_bounds__(256, 1) void feat_rows_kernel(float* __restrict__ Xall, const bf16* __restrict__ pack,
                                                           int S, int T, int M, float eps) {
  __shared__ __attribute__((aligned(16))) bf16 wbuf[2 * FR_BUF_EL];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n = lane & 15, g = lane >> 4;
  const int row = blockIdx.x * 4 + wave;  // row over the batch: member row / S, table row row % S
  const bool rowok = row < M * S;  // wave-uniform; a wave past the last row recomputes it and stores nothing
  const int rc = rowok ? row : M * S - 1;
  const int mem = rc / S, sr = rc - mem * S;
  const int64_t SE = (int64_t)S * FR_E;
  float* __restrict__ X = Xall + (int64_t)mem * T * SE;

  // ---- weight pack staging (pieces [0, 9*256): QKV rows, [9*256, 12*256): Wout rows)
  u32x4 pf[FR_PIECES];
  auto fetch = [&](int h) {
    const bf16* src = pack + (int64_t)h * FEAT_PACK_HEAD;
#pragma unroll
    for (int j = 0; j < FR_PIECES; ++j) pf[j] = *(const u32x4*)(src + (tid + 256 * j) * 8);
  };
  auto stash = [&](int buf) {
    bf16* b = wbuf + buf * FR_BUF_EL;
#pragma unroll
    for (int j = 0; j < FR_PIECES; ++j) {
      const int e = (tid + 256 * j) * 8;
      if (j < FR_QKV_PIECES) {
        *(u32x4*)(b + (e / FR_E) * FR_QKV_ST + e % FR_E) = pf[j];
      } else {
        const int e2 = e - 96 * FR_E;
        *(u32x4*)(b + FR_QKV_EL + (e2 >> 5) * FR_OUT_ST + (e2 & 31)) = pf[j];
      }
    }
  };

  fetch(0);
  // ---- the row's tokens as bf16 fragments (padding tokens t >= T are zero)
  bf16x8 xf[NT][FR_E / 32];
#pragma unroll
  for (int tt = 0; tt < NT; ++tt) {
    const int t = 16 * tt + n;
    const float* xr = X + (int64_t)(t < T ? t : 0) * SE + (int64_t)sr * FR_E + 8 * g;
#pragma unroll
    for (int ks = 0; ks < FR_E / 32; ++ks) {
      f32x4 lo = *(const f32x4*)(xr + 32 * ks), hi = *(const f32x4*)(xr + 32 * ks + 4);
      if (t >= T) lo = hi = f32x4{0.f, 0.f, 0.f, 0.f};
      xf[tt][ks] = cat8(lo, hi);
    }
  }
  stash(0);
  __syncthreads();

  f32x4 y[FR_E / 16][NT];
#pragma unroll
  for (int f = 0; f < FR_E / 16; ++f)
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) y[f][tt] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int h = 0; h < FR_H; ++h) {
    if (h + 1 < FR_H) fetch(h + 1);
    const bf16* wq = wbuf + (h & 1) * FR_BUF_EL;  // [96][FR_QKV_ST]: Q (permuted) | K (permuted) | V
    const bf16* wo = wq + FR_QKV_EL;              // [192][FR_OUT_ST]: Wout[:, head cols permuted]

    // ---- Q^T, K^T (C^T tiles) and V (C tiles) of the row, K = 192 in 6 steps
    f32x4 qa[2][NT], ka[2][NT], va[2][NT];
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
      for (int tt = 0; tt < NT; ++tt) qa[f][tt] = ka[f][tt] = va[f][tt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < FR_E / 32; ++ks) {
      bf16x8 wqf[2], wkf[2], wvf[2];
#pragma unroll
      for (int f = 0; f < 2; ++f) {
        wqf[f] = *(const bf16x8*)(wq + (16 * f + n) * FR_QKV_ST + 32 * ks + 8 * g);
        wkf[f] = *(const bf16x8*)(wq + (32 + 16 * f + n) * FR_QKV_ST + 32 * ks + 8 * g);
        wvf[f] = *(const bf16x8*)(wq + (64 + 16 * f + n) * FR_QKV_ST + 32 * ks + 8 * g);
      }
#pragma unroll
      for (int tt = 0; tt < NT; ++tt)
#pragma unroll
        for (int f = 0; f < 2; ++f) {
          qa[f][tt] = mfma16(wqf[f], xf[tt][ks], qa[f][tt]);
          ka[f][tt] = mfma16(wkf[f], xf[tt][ks], ka[f][tt]);
          va[f][tt] = mfma16(xf[tt][ks], wvf[f], va[f][tt]);
        }
    }
    bf16x8 qf[NT], kf[NT];
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) qf[tt] = cat8(qa[0][tt], qa[1][tt]), kf[tt] = cat8(ka[0][tt], ka[1][tt]);
    constexpr int NKP = (NT + 1) / 2;  // key-tile pairs (K = 32 keys per P.V MFMA)
    bf16x8 vfr[2][NKP];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int kp = 0; kp < NKP; ++kp)
        vfr[mt][kp] = cat8(va[mt][2 * kp], 2 * kp + 1 < NT ? va[mt][2 * kp + 1] : f32x4{0.f, 0.f, 0.f, 0.f});

#if defined(FR_DBG) && FR_DBG == 1  // diagnostics: no attention (O := Q)
    bf16x8 of[NT];
#pragma unroll
    for (int qt = 0; qt < NT; ++qt) of[qt] = qf[qt] + kf[qt] + vfr[0][0];
#else
    // ---- S^T[key][query] = K Q^T (scores already in log2 units), softmax over keys
    f32x4 st[NT][NT];
#pragma unroll
    for (int kt = 0; kt < NT; ++kt)
#pragma unroll
      for (int qt = 0; qt < NT; ++qt) st[kt][qt] = mfma16(kf[kt], qf[qt], f32x4{0.f, 0.f, 0.f, 0.f});
    float inv[NT];
#pragma unroll
    for (int qt = 0; qt < NT; ++qt) {
      float m = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < NT; ++kt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if (16 * kt + 4 * g + i >= T) st[kt][qt][i] = -INFINITY;
          m = fmaxf(m, st[kt][qt][i]);
        }
      m = max_rows4(m);
      float sum = 0.f;
#pragma unroll
      for (int kt = 0; kt < NT; ++kt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float e = __builtin_amdgcn_exp2f(st[kt][qt][i] - m);
          st[kt][qt][i] = e;
          sum += e;
        }
      inv[qt] = __builtin_amdgcn_rcpf(sum_rows4(sum));
    }
    // ---- O^T[d][query] = V^T P^T (P^T from the S^T accumulators, same permuted key order)
    f32x4 oa[2][NT];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int qt = 0; qt < NT; ++qt) oa[mt][qt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kp = 0; kp < NKP; ++kp)
#pragma unroll
      for (int qt = 0; qt < NT; ++qt) {
        const bf16x8 pb = cat8(st[2 * kp][qt], 2 * kp + 1 < NT ? st[2 * kp + 1][qt] : f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) oa[mt][qt] = mfma16(vfr[mt][kp], pb, oa[mt][qt]);
      }
    // ---- Y^T += Wout_h . O^T (normalised O^T as the B operand)
    bf16x8 of[NT];
#pragma unroll
    for (int qt = 0; qt < NT; ++qt) of[qt] = cat8(oa[0][qt], oa[1][qt], inv[qt]);
#endif
#pragma unroll
    for (int f = 0; f < FR_E / 16; ++f) {
      const bf16x8 wof = *(const bf16x8*)(wo + (16 * f + n) * FR_OUT_ST + 8 * g);
#pragma unroll
      for (int tt = 0; tt < NT; ++tt) y[f][tt] = mfma16(wof, of[tt], y[f][tt]);
    }
    if (h + 1 < FR_H) stash((h + 1) & 1);  // the buffer head h-1 read; every wave passed that barrier
    __syncthreads();
  }

  // ---- residual + LayerNorm per token (lane = token n of tile tt, 48 of its 192 features)
#pragma unroll
  for (int tt = 0; tt < NT; ++tt) {
    const int t = 16 * tt + n;
    const bool valid = rowok && t < T;
    float* xr = X + (int64_t)(t < T ? t : 0) * SE + (int64_t)sr * FR_E + 4 * g;
    float sm = 0.f;
#pragma unroll
    for (int f = 0; f < FR_E / 16; ++f) {
      const f32x4 xv = *(const f32x4*)(xr + 16 * f);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        y[f][tt][i] += xv[i];
        sm += y[f][tt][i];
      }
    }
    const float mean = sum_rows4(sm) * (1.0f / FR_E);
    float q = 0.f;
#pragma unroll
    for (int f = 0; f < FR_E / 16; ++f)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float dl = y[f][tt][i] - mean;
        q += dl * dl;
      }
    const float rs = 1.0f / sqrtf(sum_rows4(q) * (1.0f / FR_E) + eps);
    if (valid) {
#pragma unroll
      for (int f = 0; f < FR_E / 16; ++f) {
        f32x4 ov;
#pragma unroll
        for (int i = 0; i < 4; ++i) ov[i] = (y[f][tt][i] - mean) * rs;
        *(f32x4*)(xr + 16 * f) = ov;
      }
    }
  }
}

}  // namespace

hipError_t launch_feat_rows(float* X, const void* pack, int S, int T, int M, int E, int H, float eps,
                            hipStream_t st) {
  if (S <= 0 || M <= 0) return hipSuccess;
  if (E != FR_E || H != FR_H || T < 1 || T > 64) return hipErrorInvalidValue;
  const dim3 grid((M * S + 3) / 4), block(256);
  const bf16* pk = (const bf16*)pack;
  if (T <= 16) hipLaunchKernelGGL(feat_rows_kernel<1>, grid, block, 0, st, X, pk, S, T, M, eps);
  else if (T <= 32) hipLaunchKernelGGL(feat_rows_kernel<2>, grid, block, 0, st, X, pk, S, T, M, eps);
  else if (T <= 48) hipLaunchKernelGGL(feat_rows_kernel<3>, grid, block, 0, st, X, pk, S, T, M, eps);
  else hipLaunchKernelGGL(feat_rows_kernel<4>, grid, block, 0, st, X, pk, S, T, M, eps);
  return hipGetLastError();
}

}  // namespace mmpfn
