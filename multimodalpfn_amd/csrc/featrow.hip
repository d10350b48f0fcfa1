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
//                      operand (K-step h) of Y^T = Wout . O^T with Wout's columns permuted alike;
//                      the six heads' fragments are kept (6*NT regs) and the out-projection runs
//                      once after the last head, so no 192-wide accumulator lives across heads
//   Y^T accumulators  lane holds Y^T[feature 16f+4g+i][token n]: residual + LayerNorm per token
//                      with the 48 features of a lane reduced across the 4 lane groups.
// The softmax scale log2(e)/sqrt(32) is folded into Wq (exp2 on the scores).
// Only the weights move: they are stored as LDS images (capi.cpp pack_feat_rows: 416-B rows,
// so conflict-free ds_read_b128) and copied global -> LDS by LDS-DMA (global_load_lds, 1 KB
// per wave-instruction, no staging registers): per head a 39 KB QKV slice, double buffered,
// the next head's in flight during the current head; the 78 KB out-projection image over both
// buffers at the end.  80 KB of LDS and <= 256 VGPRs per 4-row block: two blocks per CU.
// Per row: 6*(18*NT + NT^2 + 2*NT*ceil(NT/2)) + 72*NT MFMAs; HBM traffic = X read + written once.
//
// F16 (PREC_F16: the state X is fp16, the reference's autocast dtype): the row's X^T fragments are
// loaded as they are stored (16-B loads, no conversion) and are the exact residual, so X is read once;
// the out-projection image's rows are permuted (capi.cpp: pack_feat_rows res_perm) so that Y^T tile f
// row 4g+i is feature 32(f>>1) + 8g + 4(f&1) + i -- the features of the lane's X fragments -- and
// the normalised row is stored as 16-B pieces of 8 features.
#include <type_traits>

#include "common.h"
#include "kernels.h"

namespace mmpfn {

namespace {

constexpr int FR_E = 192;                        // model width
constexpr int FR_H = 6;                          // heads
constexpr int FR_ST = FEAT_IMG_STRIDE;           // bf16 row stride of every LDS image (416 B)
constexpr int FR_QKV_IMG = 96 * FR_ST;           // one head's QKV image: 19968 bf16 = 39 KB
constexpr int FR_PIECES = FR_QKV_IMG * 2 / 1024; // 1-KB DMA pieces per QKV image (39)

template <typename X8>
__device__ __forceinline__ X8 cat8(const f32x4& a, const f32x4& b, float s = 1.0f) {
  typedef decltype(X8{}[0]) T;
  X8 r;
#pragma unroll
  for (int i = 0; i < 4; ++i) r[i] = (T)(a[i] * s), r[4 + i] = (T)(b[i] * s);
  return r;
}

typedef __attribute__((address_space(3))) void lds_void;

// one 1-KB LDS-DMA piece in the saddr form: lane i's 16 B at sbase + voff land at LDS m0 + 16 i (a scalar base per
// piece and one offset VGPR for all of them; the builtin's 64-bit VGPR address per piece cost ~19 VGPRs at the
// kernel's register peak).  m0: clang keeps it reserved and ignores the clobber (-Winline-asm); test_codegen checks
// that every m0 use in the kernels is one of these issues.
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void fr_dma16(uint32_t voff, const void* sbase, unsigned lds_dst) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sbase), "s"(lds_dst)
               : "memory", "m0");
}
#pragma clang diagnostic pop

template <int NT, bool F16>
__global__ __launch_bounds__(256, NT <= 3 ? 2 : 1) void feat_rows_kernel(void* __restrict__ Xv,
                                                                         const void* __restrict__ packv, int S, int T,
                                                                         int M, float eps) {
  typedef typename Op16<F16>::x8 X8;
  typedef std::conditional_t<F16, f16, float> XT;  // state element
  typedef typename Op16<F16>::t WT;
  const WT* __restrict__ pack = (const WT*)packv;
  __shared__ __attribute__((aligned(1024))) WT wbuf[2 * FR_QKV_IMG];
  // (wave in an SGPR: the LDS-DMA piece addresses below are then a scalar base + the lane's 16-B offset, the
  // saddr form, instead of one 64-bit VGPR address per piece -- 10 pieces a head, ~19 VGPRs at the peak)
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n = lane & 15, g = lane >> 4;
  const int row = blockIdx.x * 4 + wave;  // row over the batch: member row / S, table row row % S
  const bool rowok = row < M * S;  // wave-uniform; a wave past the last row recomputes it and stores nothing
  const int rc = rowok ? row : M * S - 1;
  const int mem = rc / S, sr = rc - mem * S;
  const int64_t SE = (int64_t)S * FR_E;
  XT* __restrict__ X = (XT*)Xv + (int64_t)mem * T * SE;

  // LDS-DMA of `pieces` KB from src (global) to dst (LDS), KB piece p by wave p % 4
  // (non-dependent pointer types: a builtin call on a template-dependent type is checked at instantiation,
  // where the host pass cannot resolve it, and the kernel's host stub is then silently dropped)
  const uint32_t dvoff = lane * 16;
  // the asm DMA issues are invisible to the compiler's waitcnt pass: each barrier that publishes an image waits
  // for this wave's pieces itself (vmcnt counts them with the wave's other global loads)
  auto dma_wait = []() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); };
  auto lds_u32 = [](const void* p) { return (unsigned)(uintptr_t)(lds_void*)p; };
  auto dma = [&](const void* srcv, void* dstv, int pieces) {
    const char* src = (const char*)srcv;
    const unsigned dst = lds_u32(dstv);
    for (int p = wave; p < pieces; p += 4)
      fr_dma16(dvoff, src + p * 1024, __builtin_amdgcn_readfirstlane(dst + p * 1024));
  };

  // the same copy one piece at a time: piece i of this wave (wave + 4 i), clamped to the last piece so that
  // the call is branch-free (a clamped piece rewrites the last piece's bytes with the same data)
  auto dma_piece = [&](const void* srcv, void* dstv, int i) {
    const int p = min(wave + 4 * i, FR_PIECES - 1);
    fr_dma16(dvoff, (const char*)srcv + p * 1024, __builtin_amdgcn_readfirstlane(lds_u32(dstv) + p * 1024));
  };
#ifndef FR_DMA_SPREAD
#define FR_DMA_SPREAD 1
#endif
  constexpr int FR_PPW = (FR_PIECES + 3) / 4;  // pieces per wave (10)
  constexpr bool SPREAD = FR_DMA_SPREAD && F16;  // the bf16 form: +16 spilled registers, not spread

  dma(pack, wbuf, FR_PIECES);  // head 0 -> buffer 0
  // row addresses: a wave-uniform row base and a 32-bit lane offset per token tile (the saddr form: one VGPR per
  // tile where a 64-bit address per tile, live to the final stores, cost spills); lane offset = token t, features 8 g
  const char* const xrow = (const char*)(X + (int64_t)sr * FR_E);
  uint32_t xoff[NT];
#pragma unroll
  for (int tt = 0; tt < NT; ++tt) {
    const int t = 16 * tt + n;
    xoff[tt] = (uint32_t)(((tt == NT - 1 && t >= T ? 0 : t) * SE + 8 * g) * sizeof(XT));
  }
  // ---- the row's tokens as bf16 fragments (padding tokens t >= T are zero)
  X8 xf[NT][FR_E / 32];
#pragma unroll
  for (int tt = 0; tt < NT; ++tt) {
    const int t = 16 * tt + n;
    const bool pad = tt == NT - 1 && t >= T;  // only the last tile holds padding (T > 16 (NT - 1))
#pragma unroll
    for (int ks = 0; ks < FR_E / 32; ++ks) {
      if constexpr (F16) {
        xf[tt][ks] = *(const f16x8*)(xrow + xoff[tt] + 64 * ks);
        if (pad) xf[tt][ks] = f16x8{};
      } else {
        const char* xr = xrow + xoff[tt] + 128 * ks;
        f32x4 lo = *(const f32x4*)xr, hi = *(const f32x4*)(xr + 16);
        if (pad) lo = hi = f32x4{0.f, 0.f, 0.f, 0.f};
        xf[tt][ks] = cat8<X8>(lo, hi);
      }
    }
  }
  dma_wait();
  __syncthreads();

  X8 of[FR_H][NT];  // O^T fragments of every head (K-step h of the out-projection)
#pragma unroll
  for (int h = 0; h < FR_H; ++h) {
    // the next image: head h+1's QKV, or after the last head the out-projection image's first half (buffer 0
    // is free); FR_DMA_SPREAD issues it one piece per k-step of the projections below instead of as one burst
    // at the head's start (an LDS-DMA's issue cost grows with the other issues of its phase,
    // MI355X_MICROARCH.md); the end-of-head barrier retires it either way
    const WT* nsrc = h + 1 < FR_H ? pack + (h + 1) * FR_QKV_IMG : pack + FR_H * FR_QKV_IMG;
    WT* ndst = h + 1 < FR_H ? wbuf + ((h + 1) & 1) * FR_QKV_IMG : wbuf;
    if constexpr (!SPREAD) dma(nsrc, ndst, FR_PIECES);
    const WT* wq = wbuf + (h & 1) * FR_QKV_IMG;  // [96][FR_ST]: Q (permuted) | K (permuted) | V

    // ---- Q^T, K^T (C^T tiles) of the row, K = 192 in 6 steps (V after, to bound live registers)
    X8 qf[NT], kf[NT];
    // Q then K, one set of 2 NT accumulators live at a time (both at once: 54 / 44 spills in the fp16 / bf16
    // forms vs 46 / 24, and 2.5 / 4.5 % slower, profiles/r04/ab_feat_rows_qk_split.txt)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      f32x4 qa[2][NT];
#pragma unroll
      for (int f = 0; f < 2; ++f)
#pragma unroll
        for (int tt = 0; tt < NT; ++tt) qa[f][tt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < FR_E / 32; ++ks) {
        X8 wqf[2];
#pragma unroll
        for (int f = 0; f < 2; ++f) wqf[f] = *(const X8*)(wq + (32 * j + 16 * f + n) * FR_ST + 32 * ks + 8 * g);
#pragma unroll
        for (int tt = 0; tt < NT; ++tt)
#pragma unroll
          for (int f = 0; f < 2; ++f) qa[f][tt] = mfma16x(wqf[f], xf[tt][ks], qa[f][tt]);
        if constexpr (SPREAD) {  // pieces 0 .. 9 after the Q and K k-steps 0 .. 4 of each
          if (ks < FR_PPW / 2) dma_piece(nsrc, ndst, j * (FR_PPW / 2) + ks);
        }
      }
#pragma unroll
      for (int tt = 0; tt < NT; ++tt) (j == 0 ? qf[tt] : kf[tt]) = cat8<X8>(qa[0][tt], qa[1][tt]);
      __builtin_amdgcn_sched_barrier(0);
    }
    __builtin_amdgcn_sched_barrier(0);  // phases in order: bounds the live registers (2 waves / SIMD)
    // ---- V (C tiles: lane = head dim, 4 consecutive tokens) -> V^T A fragments per key-tile pair
    constexpr int NKP = (NT + 1) / 2;  // key-tile pairs (K = 32 keys per P.V MFMA)
    X8 vfr[2][NKP];
    {
      f32x4 va[2][NT];
#pragma unroll
      for (int f = 0; f < 2; ++f)
#pragma unroll
        for (int tt = 0; tt < NT; ++tt) va[f][tt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < FR_E / 32; ++ks) {
        X8 wvf[2];
#pragma unroll
        for (int f = 0; f < 2; ++f) wvf[f] = *(const X8*)(wq + (64 + 16 * f + n) * FR_ST + 32 * ks + 8 * g);
#pragma unroll
        for (int tt = 0; tt < NT; ++tt)
#pragma unroll
          for (int f = 0; f < 2; ++f) va[f][tt] = mfma16x(xf[tt][ks], wvf[f], va[f][tt]);
      }
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int kp = 0; kp < NKP; ++kp)
          vfr[mt][kp] = cat8<X8>(va[mt][2 * kp], 2 * kp + 1 < NT ? va[mt][2 * kp + 1] : f32x4{0.f, 0.f, 0.f, 0.f});
    }
    __builtin_amdgcn_sched_barrier(0);

    // ---- per query tile: S^T[key][query] = K Q^T (log2 units), softmax over keys, O^T = V^T P^T
#pragma unroll
    for (int qt = 0; qt < NT; ++qt) {
      f32x4 st[NT];
#pragma unroll
      for (int kt = 0; kt < NT; ++kt) st[kt] = mfma16x(kf[kt], qf[qt], f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
      for (int i = 0; i < 4; ++i)  // only the last key tile holds padding keys (T > 16*(NT-1))
        if (16 * (NT - 1) + 4 * g + i >= T) st[NT - 1][i] = -INFINITY;
      float m = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < NT; ++kt)
#pragma unroll
        for (int i = 0; i < 4; ++i) m = fmaxf(m, st[kt][i]);
      m = max_rows4(m);
      float sum = 0.f;
#pragma unroll
      for (int kt = 0; kt < NT; ++kt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float e = __builtin_amdgcn_exp2f(st[kt][i] - m);
          st[kt][i] = e;
          sum += e;
        }
      const float inv = __builtin_amdgcn_rcpf(sum_rows4(sum));
      f32x4 oa[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int kp = 0; kp < NKP; ++kp) {
        const X8 pb = cat8<X8>(st[2 * kp], 2 * kp + 1 < NT ? st[2 * kp + 1] : f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) oa[mt] = mfma16x(vfr[mt][kp], pb, oa[mt]);
      }
      of[h][qt] = cat8<X8>(oa[0], oa[1], inv);
      __builtin_amdgcn_sched_barrier(0);
    }
    dma_wait();  // the next image landed (every wave's pieces: the barrier below); this head's buffer is free
    __syncthreads();
  }
  // second half of the out-projection image (buffer 1, read by head 5 until the barrier above)
  dma(pack + FR_H * FR_QKV_IMG + FR_QKV_IMG, wbuf + FR_QKV_IMG, FR_PIECES);
  // (running token tile 0's output features 0 .. 95, buffer 0's rows, before this barrier measured neutral:
  // 101.9 / 102.4 vs 101.3 / 101.9 µs, profiles/r04/ab_feat_rows_dma_spread.txt)
  dma_wait();
  __syncthreads();

  // ---- per token tile: Y^T = Wout . O^T over K = 192 (K-step h = head h), image [192][FR_ST],
  //      then residual + LayerNorm per token (lane = token n, 48 of its 192 features)
#pragma unroll
  for (int tt = 0; tt < NT; ++tt) {
    f32x4 y[FR_E / 16];
#pragma unroll
    for (int f = 0; f < FR_E / 16; ++f) {
      y[f] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int h = 0; h < FR_H; ++h)
        y[f] = mfma16x(*(const X8*)(wbuf + (16 * f + n) * FR_ST + 32 * h + 8 * g), of[h][tt], y[f]);
    }
    const int t = 16 * tt + n;
    const bool pad = tt == NT - 1 && t >= T;
    const bool valid = rowok && !pad;
    // fp32 state: the residual / output pieces are 4 features at 16 f + 4 g (the Y^T rows of the lane)
    char* const xr = (char*)xrow + xoff[tt] - 16 * g;
    float sm = 0.f;
    if constexpr (F16) {  // the residual is the lane's own X fragments (image rows permuted to match)
#pragma unroll
      for (int f = 0; f < FR_E / 16; ++f)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          y[f][i] += (float)xf[tt][f >> 1][4 * (f & 1) + i];
          sm += y[f][i];
        }
    } else {
#pragma unroll
      for (int f = 0; f < FR_E / 16; ++f) {
        const f32x4 xv = *(const f32x4*)(xr + 64 * f);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          y[f][i] += xv[i];
          sm += y[f][i];
        }
      }
    }
    const float mean = sum_rows4(sm) * (1.0f / FR_E);
    float q = 0.f;
#pragma unroll
    for (int f = 0; f < FR_E / 16; ++f)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float dl = y[f][i] - mean;
        q += dl * dl;
      }
    const float rs = 1.0f / sqrtf(sum_rows4(q) * (1.0f / FR_E) + eps);
    if (valid) {
      if constexpr (F16) {  // features 32k + 8g .. +7 from tiles 2k, 2k+1: one 16-B store each
#pragma unroll
        for (int k = 0; k < FR_E / 32; ++k) {
          f16x8 ov;
#pragma unroll
          for (int i = 0; i < 4; ++i)
            ov[i] = (f16)((y[2 * k][i] - mean) * rs), ov[4 + i] = (f16)((y[2 * k + 1][i] - mean) * rs);
          *(f16x8*)(xrow + xoff[tt] + 64 * k) = ov;
        }
      } else {
#pragma unroll
        for (int f = 0; f < FR_E / 16; ++f) {
          f32x4 ov;
#pragma unroll
          for (int i = 0; i < 4; ++i) ov[i] = (y[f][i] - mean) * rs;
          *(f32x4*)(xr + 64 * f) = ov;
        }
      }
    }
  }
}

template <bool F16>
hipError_t launch_fr(void* X, const void* pk, int S, int T, int M, float eps, hipStream_t st) {
  const dim3 grid((M * S + 3) / 4), block(256);
  if (T <= 16) hipLaunchKernelGGL((feat_rows_kernel<1, F16>), grid, block, 0, st, X, pk, S, T, M, eps);
  else if (T <= 32) hipLaunchKernelGGL((feat_rows_kernel<2, F16>), grid, block, 0, st, X, pk, S, T, M, eps);
  else if (T <= 48) hipLaunchKernelGGL((feat_rows_kernel<3, F16>), grid, block, 0, st, X, pk, S, T, M, eps);
  else hipLaunchKernelGGL((feat_rows_kernel<4, F16>), grid, block, 0, st, X, pk, S, T, M, eps);
  return hipGetLastError();
}
}  // namespace

hipError_t launch_feat_rows(void* X, const void* pack, int S, int T, int M, int E, int H, float eps, hipStream_t st,
                            bool f16) {
  if (S <= 0 || M <= 0) return hipSuccess;
  if (E != FR_E || H != FR_H || T < 1 || T > 64) return hipErrorInvalidValue;
  return f16 ? launch_fr<true>(X, pack, S, T, M, eps, st) : launch_fr<false>(X, pack, S, T, M, eps, st);
}

}  // namespace mmpfn
