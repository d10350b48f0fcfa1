// Row-resident MLP sublayer for gfx950 (bf16 performance mode):
//   X <- LayerNorm(X + GELU(X W1^T) W2^T)           (mlp.py:93-104, layer.py:437-455)
// optionally fused with the item-attention out-projection before it (RES):
//   X <- LayerNorm(X + O Wout^T) first              (layer.py:341-379,437-455)
//
// Each wave owns 32 rows (tokens) for the whole sublayer and keeps them in registers:
//   * its rows of X, as bf16 B-operand fragments (A^T), loaded once from HBM -- in the lane
//     layout of a Y^T accumulator (lane = row, features 16f + 4g + i), W1's K order permuted
//     to match (capi.cpp pack_mlp1_perm), so RES can feed its LayerNorm output straight in;
//   * the hidden activations of a 32-wide hidden chunk, computed transposed
//     (H^T = W1c . A^T) so the accumulator of one 16x16 tile pair is, lane for lane, the B
//     operand of the down projection (Y^T += W2c . H^T) once the chunk's K order is
//     permuted (pos 8g+j <-> hidden 4g+j / 16+4g+j-4; W2 stored so, capi.cpp pack_mlp2_perm);
//   * the 192 x 32 output accumulator Y^T, initialised with the fp32 residual itself (X, or the
//     fused prologue's X'), so the residual never leaves registers; then LayerNorm across lanes.
// Software pipeline over hidden chunks c (branch-free body, last chunk peeled): GELU(H(c)) on
// the VALU beside the MFMAs of H(c+1), then Y^T += W2c . GELU(H(c)); one barrier per chunk.
// Only the weights move through LDS: a 128-row block (4 waves) shares each chunk; W1 of chunk
// c+2 and W2 of chunk c+1 are loaded into registers during chunk c and written to their LDS
// slots after it (two slots each, 62 KB per block: two blocks per CU).  LDS rows of 416 B
// (W1) and 96 B (W2) keep the ds_read_b128 fragment reads conflict-free.
#include "common.h"
#include "kernels.h"

namespace mmpfn {

namespace {

constexpr int RE = 192;                    // model width
constexpr int RHC = 32;                    // hidden chunk
constexpr int W1ST = RE + 16;              // W1 chunk LDS row stride (bf16): 416 B
constexpr int W2ST = RHC + 16;             // W2 chunk LDS row stride (bf16): 96 B
constexpr int W1EL = RHC * W1ST;           // 6656
constexpr int W2EL = RE * W2ST;            // 9216
constexpr int P1 = RHC * RE / 8 / 256;     // 16-B W1 pieces per thread and chunk (3)
constexpr int P2 = RE * RHC / 8 / 256;     // 16-B W2 pieces per thread and chunk (3)

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// TT = 16-row tiles per wave: 2 (32 rows, two waves per SIMD, accumulators in VGPRs) or 4 (64 rows,
// one wave per SIMD with the 192 x 64 Y^T accumulator in AGPRs -- half the LDS weight reads per row,
// but measured 15% slower: one wave cannot hide the LDS / GELU latency the second wave covers)
template <int TT, bool RES>
__global__ __launch_bounds__(256, TT == 2 ? 2 : 1) void mlp_rows_kernel(float* __restrict__ X,
                                                                       const bf16* __restrict__ W1,
                                                                       const bf16* __restrict__ W2p, int M, int Fh,
                                                                       float eps, const bf16* __restrict__ O,
                                                                       const bf16* __restrict__ Wout) {
  constexpr int RROWS = 4 * 16 * TT;  // rows per block
  __shared__ __attribute__((aligned(16))) bf16 lds[2 * W1EL + 2 * W2EL];
  bf16* const w1s = lds;
  bf16* const w2s = lds + 2 * W1EL;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const int64_t m0 = (int64_t)blockIdx.x * RROWS + wave * 16 * TT;
  const int nchunks = Fh / RHC;

  // register staging: piece p of W1 chunk c = row c*32 + p/24, 16-B column p%24;
  // piece q of W2 chunk c = row q/4, 16-B column q%4 of the chunk's 32 permuted columns
  u32x4 r1[P1], r2[P2];
  auto fetch1 = [&](int c) {
#pragma unroll
    for (int j = 0; j < P1; ++j) {
      const int p = tid + 256 * j;
      r1[j] = *(const u32x4*)(W1 + (int64_t)(c * RHC + p / 24) * RE + (p % 24) * 8);
    }
  };
  auto fetch2 = [&](int c) {
#pragma unroll
    for (int j = 0; j < P2; ++j) {
      const int q = tid + 256 * j;
      r2[j] = *(const u32x4*)(W2p + (int64_t)(q >> 2) * Fh + c * RHC + (q & 3) * 8);
    }
  };
  auto stash1 = [&](int slot) {
#pragma unroll
    for (int j = 0; j < P1; ++j) {
      const int p = tid + 256 * j;
      *(u32x4*)(w1s + slot * W1EL + (p / 24) * W1ST + (p % 24) * 8) = r1[j];
    }
  };
  auto stash2 = [&](int slot) {
#pragma unroll
    for (int j = 0; j < P2; ++j) {
      const int q = tid + 256 * j;
      *(u32x4*)(w2s + slot * W2EL + (q >> 2) * W2ST + (q & 3) * 8) = r2[j];
    }
  };

  // ---- the wave's rows as B fragments in the Y^T lane layout: lane (row 16tt + fr, group fg)
  //      holds features 16f + 4fg + i; K position 32ks + 8fg + j <-> feature of tile f = 2ks + j/4
  bf16x8 af[TT][RE / 32];
  f32x4 y[RE / 16][TT];
  auto to_af = [&](int tt) {
#pragma unroll
    for (int ks = 0; ks < RE / 32; ++ks) {
      bf16x8 b;
#pragma unroll
      for (int i = 0; i < 4; ++i) b[i] = (bf16)y[2 * ks][tt][i], b[4 + i] = (bf16)y[2 * ks + 1][tt][i];
      af[tt][ks] = b;
    }
  };
  if constexpr (RES) {
    // X <- LayerNorm(X + O . Wout^T): Wout [192 out][192 in] staged in two 96-row halves through
    // the (still unused) weight slots, C^T tiles (lane = row) as in rowgemm_resln
    bf16x8 ao[TT][RE / 32];
#pragma unroll
    for (int tt = 0; tt < TT; ++tt) {
      const int64_t m = min(m0 + tt * 16 + fr, (int64_t)M - 1);
#pragma unroll
      for (int ks = 0; ks < RE / 32; ++ks) ao[tt][ks] = *(const bf16x8*)(O + m * RE + ks * 32 + fg * 8);
    }
#pragma unroll
    for (int f = 0; f < RE / 16; ++f)
#pragma unroll
      for (int tt = 0; tt < TT; ++tt) y[f][tt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      constexpr int PC = 96 * (RE / 8) / 256;  // 16-B pieces per thread (9)
#pragma unroll
      for (int r = 0; r < 3; ++r) {            // three rounds of 3 pieces: bounded staging registers
        u32x4 st[PC / 3];
#pragma unroll
        for (int j = 0; j < PC / 3; ++j) {
          const int pc = tid + 256 * (r * (PC / 3) + j);
          st[j] = *(const u32x4*)(Wout + (int64_t)(96 * half + pc / 24) * RE + (pc % 24) * 8);
        }
#pragma unroll
        for (int j = 0; j < PC / 3; ++j) {
          const int pc = tid + 256 * (r * (PC / 3) + j);
          *(u32x4*)(lds + (pc / 24) * W1ST + (pc % 24) * 8) = st[j];
        }
      }
      __syncthreads();
#pragma unroll
      for (int ks = 0; ks < RE / 32; ++ks)
#pragma unroll
        for (int fl = 0; fl < 6; ++fl) {
          const bf16x8 w = *(const bf16x8*)(lds + (fl * 16 + fr) * W1ST + ks * 32 + fg * 8);
#pragma unroll
          for (int tt = 0; tt < TT; ++tt) y[6 * half + fl][tt] = mfma16(w, ao[tt][ks], y[6 * half + fl][tt]);
        }
      __syncthreads();
    }
    // residual + LayerNorm (layer.py:437-455), X' written back (the MLP's residual) and packed
#pragma unroll
    for (int tt = 0; tt < TT; ++tt) {
      const int64_t m = m0 + tt * 16 + fr;
      const bool valid = m < M;
      float* xr = X + (valid ? m : (int64_t)M - 1) * RE + fg * 4;
      float sm = 0.f;
#pragma unroll
      for (int f = 0; f < RE / 16; ++f) {
        const f32x4 xv = *(const f32x4*)(xr + f * 16);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          y[f][tt][i] += xv[i];
          sm += y[f][tt][i];
        }
      }
      const float mean = sum_rows4(sm) * (1.0f / RE);
      float q = 0.f;
#pragma unroll
      for (int f = 0; f < RE / 16; ++f)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float dl = y[f][tt][i] - mean;
          q += dl * dl;
        }
      const float inv = 1.0f / sqrtf(sum_rows4(q) * (1.0f / RE) + eps);
#pragma unroll
      for (int f = 0; f < RE / 16; ++f)
#pragma unroll
        for (int i = 0; i < 4; ++i) y[f][tt][i] = (y[f][tt][i] - mean) * inv;
      to_af(tt);
    }
    fetch1(0);
    fetch2(0);
  } else {
    fetch1(0);
    fetch2(0);
#pragma unroll
    for (int tt = 0; tt < TT; ++tt) {
      const int64_t m = min(m0 + tt * 16 + fr, (int64_t)M - 1);
      const float* xr = X + m * RE + fg * 4;
#pragma unroll
      for (int f = 0; f < RE / 16; ++f) y[f][tt] = *(const f32x4*)(xr + f * 16);
      to_af(tt);
    }
  }
  stash1(0);
  stash2(0);
  if (nchunks > 1) {
    fetch1(1);
    stash1(1);
  }
  __syncthreads();

  // H^T [32 hidden][16 TT rows] = W1c . A^T  (W1c in LDS)
  auto hmma = [&](const bf16* w1, f32x4 (&h)[2][TT]) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int tt = 0; tt < TT; ++tt) h[i][tt] = f32x4{0.f, 0.f, 0.f, 0.f};
    constexpr int PU = 2;  // k-steps of W1 fragments in flight ahead of their MFMAs (measured best of 1-3)
    bf16x8 wa[PU][2];
#pragma unroll
    for (int i = 0; i < PU; ++i)
#pragma unroll
      for (int ht = 0; ht < 2; ++ht) wa[i][ht] = *(const bf16x8*)(w1 + (ht * 16 + fr) * W1ST + i * 32 + fg * 8);
#pragma unroll
    for (int ks = 0; ks < RE / 32; ++ks) {
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int ht = 0; ht < 2; ++ht)
#pragma unroll
        for (int tt = 0; tt < TT; ++tt) h[ht][tt] = mfma16(wa[ks % PU][ht], af[tt][ks], h[ht][tt]);
      if (ks + PU < RE / 32)
#pragma unroll
        for (int ht = 0; ht < 2; ++ht)
          wa[ks % PU][ht] = *(const bf16x8*)(w1 + (ht * 16 + fr) * W1ST + (ks + PU) * 32 + fg * 8);
    }
  };
  // y holds the residual (X, or X' after the fused prologue) in fp32: the down-projection MFMAs
  // accumulate onto it, so the residual is never written out and read back
  f32x4 h[2][TT];
  hmma(w1s, h);
  // chunk 0 overwrites W1 slot 0 (with W1(2)) after its MFMAs: every wave of the block must have
  // finished reading slot 0 above first -- without this barrier a wave that lags a whole chunk
  // behind (another kernel sharing its SIMD) read half-replaced W1(0) fragments
  if (nchunks > 2) __syncthreads();

  // one chunk: slots W1(c+1) in w1s[(c+1)&1], W2(c) in w2s[c&1]; W1(c+2) -> w1s[c&1] and
  // W2(c+1) -> w2s[(c+1)&1], written after this chunk's reads; both slots were last read in
  // chunk c-1 (or, for W1(0), right before chunk 0, behind the barrier after that read)
  auto chunk = [&](int c, auto morec) {
    constexpr bool MORE = decltype(morec)::value;  // a chunk c+1 exists
#ifndef MLP_NOSTAGE
    const bool f1 = c + 2 < nchunks;
    if (f1) fetch1(c + 2);
    if (MORE) fetch2(c + 1);
#endif
    bf16x8 hb[TT];  // GELU of chunk c (VALU) beside the up-projection MFMAs of chunk c+1
#pragma unroll
    for (int tt = 0; tt < TT; ++tt) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
#ifndef MLP_NOGELU
        hb[tt][i] = (bf16)gelu_tanh_fast(h[0][tt][i]);
        hb[tt][4 + i] = (bf16)gelu_tanh_fast(h[1][tt][i]);
#else
        hb[tt][i] = (bf16)h[0][tt][i];
        hb[tt][4 + i] = (bf16)h[1][tt][i];
#endif
      }
    }
    if (MORE) hmma(w1s + ((c + 1) & 1) * W1EL, h);
    // Y^T [192][32 rows] += W2c(perm) . GELU(H^T)
    const bf16* w2 = w2s + (c & 1) * W2EL;
    {  // W2 fragments 4 tiles ahead of their MFMAs (fenced so the reads stay early; 3-6 measured)
      constexpr int PF = 4;
      bf16x8 wb[PF];
#pragma unroll
      for (int i = 0; i < PF; ++i) wb[i] = *(const bf16x8*)(w2 + (i * 16 + fr) * W2ST + fg * 8);
#pragma unroll
      for (int o = 0; o < RE / 16; ++o) {
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int tt = 0; tt < TT; ++tt) y[o][tt] = mfma16(wb[o % PF], hb[tt], y[o][tt]);
        if (o + PF < RE / 16) wb[o % PF] = *(const bf16x8*)(w2 + ((o + PF) * 16 + fr) * W2ST + fg * 8);
      }
    }
#ifndef MLP_NOSTAGE
    if (f1) stash1(c & 1);
    if (MORE) stash2((c + 1) & 1);
#endif
#ifndef MLP_NOSYNC
    __syncthreads();
#endif
  };
  for (int c = 0; c + 1 < nchunks; ++c) chunk(c, std::true_type{});
  chunk(nchunks - 1, std::false_type{});

  // residual + LayerNorm: lane = row, 48 of its 192 features (rows 16o + 4g + i of Y^T)
#pragma unroll
  for (int tt = 0; tt < TT; ++tt) {
    const int64_t m = m0 + tt * 16 + fr;
    const bool valid = m < M;
    float* xr = X + (valid ? m : (int64_t)M - 1) * RE + fg * 4;
    float s = 0.f;
#pragma unroll
    for (int o = 0; o < RE / 16; ++o)
#pragma unroll
      for (int i = 0; i < 4; ++i) s += y[o][tt][i];
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
#ifndef MLP_NOSTORE
        *(f32x4*)(xr + o * 16) = ov;
#else
        if (ov[0] == 1234.5f && ov[3] == 4321.f) xr[o] = ov[1];
#endif
      }
    }
  }
}

}  // namespace

hipError_t launch_mlp_rows(float* X, const void* W1perm, const void* W2perm, int64_t M, int E, int Fh, float eps,
                           hipStream_t st, const void* O, const void* Wout) {
  if (M <= 0) return hipSuccess;
  if (E != RE || Fh % RHC != 0) return hipErrorInvalidValue;
#ifndef MLP_TT
#define MLP_TT 2  // 4 measured slower: 202 vs 175 us per two-member launch
#endif
  constexpr int RROWS = 64 * MLP_TT;
  const dim3 grid((unsigned)((M + RROWS - 1) / RROWS)), block(256);
  if (O)
    hipLaunchKernelGGL((mlp_rows_kernel<MLP_TT, true>), grid, block, 0, st, X, (const bf16*)W1perm,
                       (const bf16*)W2perm, (int)M, Fh, eps, (const bf16*)O, (const bf16*)Wout);
  else
    hipLaunchKernelGGL((mlp_rows_kernel<MLP_TT, false>), grid, block, 0, st, X, (const bf16*)W1perm,
                       (const bf16*)W2perm, (int)M, Fh, eps, nullptr, nullptr);
  return hipGetLastError();
}

}  // namespace mmpfn
