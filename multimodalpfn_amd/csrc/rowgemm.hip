// Row-resident projection GEMMs of the item-attention sublayer for gfx950 (bf16 mode):
//   * QKV : rows of X (fp32 state) . W^T (W [N][192], N = 576 q|k|v or 192 q only),
//           scattered straight into the attention layouts Q [b][h][pos][32],
//           K [b][h][pos][32] (Npad rows) and V^T [b][h][32][Npad]  (layer.py:341-372);
//   * RES_LN : X <- LayerNorm(X + O . Wout^T)  (layer.py:437-455, no affine).
// K is the model width (192): a wave keeps its 32 rows as bf16 fragments in registers
// for the whole kernel; the block (4 waves, 128 rows) streams the weights through LDS
// (row stride 416 B: conflict-free ds_read_b128) -- QKV in 64-feature chunks, RES_LN as
// one 192 x 192 panel.  Q and K chunks are computed transposed (lane = row, 4 consecutive head dims -> one 8-byte
// store); the V panel is computed untransposed (lane = head dim, 4 consecutive rows
// -> one 8-byte store into V^T).  The RES_LN panel keeps Y^T in registers and does the
// residual + LayerNorm across lanes (in-register permlane reductions).
//
// F16 (PREC_F16): X is the fp16 state -- a wave's fragments are 16-B loads of it, no conversion --,
// the weights are fp16, Q / K are written in fp16 and V^T in bf16 (the attention's P.V runs on bf16:
// its P = exp2(s) under a fixed reference needs bf16's exponent range); RES_LN reads O (fp16) and the
// fp16 residual and uses f16_row_perm-ordered weight rows, so each lane's features are 16-B runs.
#include <type_traits>

#include "common.h"
#include "kernels.h"

namespace mmpfn {

namespace {

constexpr int GE = 192;         // K (model width) and panel width
constexpr int GROWS = 128;      // rows per block
constexpr int WST = GE + 16;    // LDS panel row stride (bf16): 416 B
constexpr int WPC = GE * GE / 8 / 256;  // 16-B panel pieces per thread (18)

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma16(f16x8 a, f16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

struct RgArgs {
  const void* A;     // fp32 / fp16 (F16) rows (QKV) or 16-bit rows (RES_LN), ld = 192
  int64_t a_rdiv, a_rmul, a_rmul2, a_roff;  // logical row m -> memory row (m/rdiv)*rmul + (m%rdiv)*rmul2 + roff
  const void* W;     // [N][192] 16-bit
  int M, N;
  // QKV scatter: b = m / a_rdiv, pos = a_roff + m % a_rdiv (Q / K 16-bit of the mode, V^T bf16)
  void *q, *k;
  bf16* vt;
  int S, Npad, H;
  // RES_LN
  void* X;
  float eps;
};

template <bool AF32, typename X8>
__device__ __forceinline__ void load_rows(const RgArgs& p, int64_t m0, int fr, int fg, X8 (&af)[2][GE / 32]) {
#pragma unroll
  for (int tt = 0; tt < 2; ++tt) {
    const int m = (int)min(m0 + tt * 16 + fr, (int64_t)p.M - 1);
    const int rd = (int)p.a_rdiv, mb = m / rd;
    const int64_t mr = (int64_t)mb * p.a_rmul + (int64_t)(m - mb * rd) * p.a_rmul2 + p.a_roff;
    if constexpr (AF32) {
      const float* xr = (const float*)p.A + mr * GE + fg * 8;
      f32x4 lo[GE / 32], hi[GE / 32];
#pragma unroll
      for (int ks = 0; ks < GE / 32; ++ks) {
        lo[ks] = *(const f32x4*)(xr + ks * 32);
        hi[ks] = *(const f32x4*)(xr + ks * 32 + 4);
      }
#pragma unroll
      for (int ks = 0; ks < GE / 32; ++ks) {
        bf16x8 b;
        b[0] = (bf16)lo[ks][0], b[1] = (bf16)lo[ks][1], b[2] = (bf16)lo[ks][2], b[3] = (bf16)lo[ks][3];
        b[4] = (bf16)hi[ks][0], b[5] = (bf16)hi[ks][1], b[6] = (bf16)hi[ks][2], b[7] = (bf16)hi[ks][3];
        af[tt][ks] = b;
      }
    } else {
      const uint16_t* xr = (const uint16_t*)p.A + mr * GE + fg * 8;
#pragma unroll
      for (int ks = 0; ks < GE / 32; ++ks) af[tt][ks] = *(const X8*)(xr + ks * 32);
    }
  }
}

// stage W rows [n0, n0 + 192) into the LDS panel (all threads; caller brackets with barriers)
__device__ __forceinline__ void stage_panel(const uint16_t* W, int n0, uint16_t* Ws, int tid) {
#pragma unroll
  for (int half = 0; half < 2; ++half) {  // two rounds of 9 pieces: bounded register footprint
    u32x4 r[WPC / 2];
#pragma unroll
    for (int j = 0; j < WPC / 2; ++j) {
      const int i = tid + 256 * (half * (WPC / 2) + j);
      r[j] = *(const u32x4*)(W + (int64_t)(n0 + i / (GE / 8)) * GE + (i % (GE / 8)) * 8);
    }
#pragma unroll
    for (int j = 0; j < WPC / 2; ++j) {
      const int i = tid + 256 * (half * (WPC / 2) + j);
      *(u32x4*)(Ws + (i / (GE / 8)) * WST + (i % (GE / 8)) * 8) = r[j];
    }
  }
}

// acc[f][tt] = panel(f) x rows(tt) over K = 192; TRANS: C^T (features x rows), else C (rows x features)
template <bool TRANS, typename X8>
__device__ __forceinline__ void panel_mma(const uint16_t* Ws, const X8 (&af)[2][GE / 32], int fr, int fg,
                                          f32x4 (&acc)[GE / 16][2]) {
#pragma unroll
  for (int f = 0; f < GE / 16; ++f) acc[f][0] = acc[f][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  // W fragments in groups of 4 feature tiles, the next group's reads issued before this
  // group's MFMAs (sched barriers keep the reads early; 2 x 4 fragments in flight)
  constexpr int NG = GE / 16 / 4;  // groups per k-step (3)
  X8 w[2][4];
#pragma unroll
  for (int i = 0; i < 4; ++i) w[0][i] = *(const X8*)(Ws + (i * 16 + fr) * WST + fg * 8);
#pragma unroll
  for (int it = 0; it < (GE / 32) * NG; ++it) {
    const int ks = it / NG, g = it % NG;
    if (it + 1 < (GE / 32) * NG) {
      const int ks1 = (it + 1) / NG, g1 = (it + 1) % NG;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        w[(it + 1) & 1][i] = *(const X8*)(Ws + ((g1 * 4 + i) * 16 + fr) * WST + ks1 * 32 + fg * 8);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) {
        if constexpr (TRANS)
          acc[g * 4 + i][tt] = mfma16(w[it & 1][i], af[tt][ks], acc[g * 4 + i][tt]);
        else
          acc[g * 4 + i][tt] = mfma16(af[tt][ks], w[it & 1][i], acc[g * 4 + i][tt]);
      }
  }
}

// QKV v2: one block per 128-row tile computes ALL N outputs (576: q|k|v, or 192: q), so X comes
// from HBM once.  W streams through LDS in 64-feature chunks (two slots, 53 KB); chunk c+2 is fetched into registers while chunk c's MFMAs run and chunk c+1 is written to
// its slot at the top of the iteration (its slot was last read before the previous barrier).
constexpr int QC = 64;                     // output features per chunk
constexpr int QCEL = QC * WST;             // chunk slot elements
constexpr int QCP = QC * GE / 8 / 256;     // 16-B pieces per thread and chunk (6)

// acc[f][tt] over K = 192 for one 64-feature chunk in LDS: the next k-step's 4 fragments are
// read before this k-step's 8 MFMAs (sched barrier keeps them early)
template <bool TRANS, typename X8>
__device__ __forceinline__ void chunk_mma(const uint16_t* W, const X8 (&af)[2][GE / 32], int fr, int fg,
                                          f32x4 (&acc)[QC / 16][2]) {
  X8 w[2][QC / 16];
#pragma unroll
  for (int f = 0; f < QC / 16; ++f) w[0][f] = *(const X8*)(W + (f * 16 + fr) * WST + fg * 8);
#pragma unroll
  for (int ks = 0; ks < GE / 32; ++ks) {
    if (ks + 1 < GE / 32)
#pragma unroll
      for (int f = 0; f < QC / 16; ++f)
        w[(ks + 1) & 1][f] = *(const X8*)(W + (f * 16 + fr) * WST + (ks + 1) * 32 + fg * 8);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int f = 0; f < QC / 16; ++f)
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) {
        if constexpr (TRANS)
          acc[f][tt] = mfma16(w[ks & 1][f], af[tt][ks], acc[f][tt]);
        else
          acc[f][tt] = mfma16(af[tt][ks], w[ks & 1][f], acc[f][tt]);
      }
  }
}

// Per-wave output staging: the chunk's C tile goes through LDS so that every global store
// writes 16 B per lane in contiguous runs -- Q / K: [32 rows][64 features] (2 KB per head
// and wave, whole 1 KB per instruction), V^T: [64 features][32 rows] (64-B runs of 32 keys).
// Blocks never straddle a column b (grid = column x row tiles), so a wave's 32 rows are
// consecutive positions starting at a multiple of 32 (+ a_roff).
constexpr int OQST = QC + 8;    // Q/K tile row stride (bf16): 144 B
constexpr int OVST = 32 + 8;    // V^T tile row stride (bf16): 80 B
constexpr int OWEL = QC * OVST; // per-wave staging elements (>= 32 * OQST)
static_assert(32 * OQST <= OWEL, "Q/K staging tile must fit");

// QKB: Q / K stored in bf16 whatever the operand type (the fp16 mode's forward: its attention runs S on bf16 MFMA)
template <bool F16, bool QKB>
__device__ __forceinline__ void qkv2_tile(const RgArgs& p, int tiles_per_b, int bid, uint16_t* Ws) {
  typedef typename Op16<F16 && !QKB>::t OT;  // Q / K element
  typedef typename Op16<F16>::x8 X8;
  typedef typename Op16<F16 && !QKB>::x4 X4;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fg = lane >> 4;
  const int rd = (int)p.a_rdiv;
  const int b = bid / tiles_per_b;
  const int l0 = (bid - b * tiles_per_b) * GROWS + wave * 32;  // wave's first row inside column b
  // all 32 of the wave's rows exist (wave-uniform): the chunk stores then run unguarded, so the loop body
  // carries no exec-mask branches; only a column's last partial tile takes the guarded stores
  const bool full = l0 + 32 <= rd;
  uint16_t* const Os = Ws + 2 * QCEL + wave * OWEL;
  const int nch = p.N / QC;
  const uint16_t* Wg = (const uint16_t*)p.W;
  u32x4 r[QCP];
  auto fetch = [&](int c) {
#pragma unroll
    for (int j = 0; j < QCP; ++j) {
      const int i = tid + 256 * j;
      r[j] = *(const u32x4*)(Wg + (int64_t)(c * QC + i / (GE / 8)) * GE + (i % (GE / 8)) * 8);
    }
  };
  auto stash = [&](int slot) {
#pragma unroll
    for (int j = 0; j < QCP; ++j) {
      const int i = tid + 256 * j;
      *(u32x4*)(Ws + slot * QCEL + (i / (GE / 8)) * WST + (i % (GE / 8)) * 8) = r[j];
    }
  };
  fetch(0);
  X8 af[2][GE / 32];
  if constexpr (F16) {  // the fp16 state is the operand: 16-B loads straight into the fragments
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      const int l = min(l0 + tt * 16 + fr, rd - 1);
      const f16* xr = (const f16*)p.A + ((int64_t)b * p.a_rmul + (int64_t)l * p.a_rmul2 + p.a_roff) * GE + fg * 8;
#pragma unroll
      for (int ks = 0; ks < GE / 32; ++ks) af[tt][ks] = *(const f16x8*)(xr + ks * 32);
    }
  } else {
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      const int l = min(l0 + tt * 16 + fr, rd - 1);
      const float* xr = (const float*)p.A + ((int64_t)b * p.a_rmul + (int64_t)l * p.a_rmul2 + p.a_roff) * GE + fg * 8;
      f32x4 lo[GE / 32], hi[GE / 32];
#pragma unroll
      for (int ks = 0; ks < GE / 32; ++ks) {
        lo[ks] = *(const f32x4*)(xr + ks * 32);
        hi[ks] = *(const f32x4*)(xr + ks * 32 + 4);
      }
#pragma unroll
      for (int ks = 0; ks < GE / 32; ++ks) {
        bf16x8 v;
        v[0] = (bf16)lo[ks][0], v[1] = (bf16)lo[ks][1], v[2] = (bf16)lo[ks][2], v[3] = (bf16)lo[ks][3];
        v[4] = (bf16)hi[ks][0], v[5] = (bf16)hi[ks][1], v[6] = (bf16)hi[ks][2], v[7] = (bf16)hi[ks][3];
        af[tt][ks] = v;
      }
    }
  }
  stash(0);
  if (nch > 1) fetch(1);
  __syncthreads();
  const int pos0 = (int)p.a_roff + l0;  // attention position of the wave's row 0
  auto run = [&](auto fullc) {
    constexpr bool FULL = decltype(fullc)::value;
    for (int c = 0; c < nch; ++c) {
      if (c + 1 < nch) stash((c + 1) & 1);
      if (c + 2 < nch) fetch(c + 2);
      const uint16_t* W = Ws + (c & 1) * QCEL;
      const int n0 = c * QC, j = n0 / GE;  // 0 q, 1 k, 2 v
      const int h0 = (n0 - j * GE) >> 5;   // first of the chunk's two heads
      f32x4 acc[QC / 16][2];
  #pragma unroll
      for (int f = 0; f < QC / 16; ++f) acc[f][0] = acc[f][1] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (j < 2) {
        chunk_mma<true>(W, af, fr, fg, acc);
        // C^T: lane = row 16tt + fr, features 16f + 4fg + i  ->  Os[row][feature]
  #pragma unroll
        for (int tt = 0; tt < 2; ++tt)
  #pragma unroll
          for (int f = 0; f < QC / 16; ++f) {
            X4 o;
            o[0] = (OT)acc[f][tt][0], o[1] = (OT)acc[f][tt][1];
            o[2] = (OT)acc[f][tt][2], o[3] = (OT)acc[f][tt][3];
            *(X4*)(Os + (tt * 16 + fr) * OQST + f * 16 + fg * 4) = o;
          }
        uint16_t* base = j == 0 ? (uint16_t*)p.q + (((int64_t)b * p.H + h0) * p.S + pos0) * 32
                                : (uint16_t*)p.k + (((int64_t)b * p.H + h0) * p.Npad + pos0) * 32;
        const int64_t hstride = (int64_t)(j == 0 ? p.S : p.Npad) * 32;
  #pragma unroll
        for (int hh = 0; hh < 2; ++hh)
  #pragma unroll
          for (int i = 0; i < 2; ++i) {
            const int row = 16 * i + (lane >> 2), cc = lane & 3;
            const u32x4 v = *(const u32x4*)(Os + row * OQST + hh * 32 + cc * 8);
            if (FULL || l0 + row < rd) *(u32x4*)(base + hh * hstride + row * 32 + cc * 8) = v;
          }
      } else {
        chunk_mma<false>(W, af, fr, fg, acc);
        // C: lane = feature 16f + fr, rows 16tt + 4fg + i  ->  Os[feature][row]
  #pragma unroll
        for (int tt = 0; tt < 2; ++tt)
  #pragma unroll
          for (int f = 0; f < QC / 16; ++f) {
            bf16x4 o;
            o[0] = (bf16)acc[f][tt][0], o[1] = (bf16)acc[f][tt][1];
            o[2] = (bf16)acc[f][tt][2], o[3] = (bf16)acc[f][tt][3];
            *(bf16x4*)(Os + (f * 16 + fr) * OVST + tt * 16 + fg * 4) = o;
          }
        uint16_t* base = (uint16_t*)p.vt + ((int64_t)b * p.H + h0) * 32 * p.Npad + pos0;
  #pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int feat = 16 * i + (lane >> 2), rr = (lane & 3) * 8;
          const u32x4 v = *(const u32x4*)(Os + feat * OVST + rr);
          uint16_t* dst = base + (int64_t)feat * p.Npad + rr;  // feature = (head - h0) * 32 + d
          if (FULL || l0 + rr + 8 <= rd) {
            *(u32x4*)dst = v;
          } else {
            typedef __attribute__((ext_vector_type(8))) unsigned short u16x8;
            const u16x8 e = __builtin_bit_cast(u16x8, v);
  #pragma unroll
            for (int k = 0; k < 8; ++k)
              if (l0 + rr + k < rd) dst[k] = e[k];
          }
        }
      }
      __syncthreads();
    }
  };
#ifndef QKV_VERSIONED
#define QKV_VERSIONED 1
#endif
  if (QKV_VERSIONED && full) run(std::true_type{});
  else run(std::false_type{});
}

// Two row sets in one launch: blocks [0, nblk1) project p's rows (the train rows: q|k|v), the
// rest p2's (the test rows: q only, a third of the chunks) -- the short test-row blocks run last
// and fill the grid's tail instead of a separate under-filled launch.
template <bool F16, bool QKB>
__global__ __launch_bounds__(256, 2) void rowgemm_qkv2_kernel(const RgArgs p, int tiles_per_b, const RgArgs p2,
                                                              int tiles2, int nblk1) {
  __shared__ __attribute__((aligned(16))) uint16_t Ws[2 * QCEL + 4 * OWEL];
  if ((int)blockIdx.x < nblk1) qkv2_tile<F16, QKB>(p, tiles_per_b, blockIdx.x, Ws);
  else qkv2_tile<F16, QKB>(p2, tiles2, blockIdx.x - nblk1, Ws);
}

// C[m] = (LN? LayerNorm(A[m]) : A[m]) . W^T + bias, A fp32 [M][192], W [N][192] bf16, C bf16 [M][N]
// (N % 64 == 0): the CAP K|V projection of the normalised mixer tokens (transformer.py:77-84) in
// one pass -- the LayerNorm (no affine; folded into W on the host) runs on the rows in registers,
// so the normalised copy never reaches HBM.  Same chunk pipeline and LDS-staged 16-B stores as
// the QKV kernel above.  vt_from >= 0: outputs [vt_from, N) go transposed per group of Mk rows
// (Mk % 32 == 0), CT [M / Mk][N - vt_from][Mk] (the CAP V^T: keys contiguous), the rest to C with
// row stride ldc.
template <typename TA>
__global__ __launch_bounds__(256, 2) void rowgemm_ln_store_kernel(const TA* __restrict__ A, const bf16* __restrict__ W,
                                                                  const float* __restrict__ bias, bf16* __restrict__ C,
                                                                  int M, int N, float eps, int do_ln, int ldc,
                                                                  bf16* __restrict__ CT, int vt_from, int Mk) {
  __shared__ __attribute__((aligned(16))) uint16_t Ws[2 * QCEL + 4 * OWEL];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const int64_t m0 = (int64_t)blockIdx.x * GROWS + wave * 32;
  uint16_t* const Os = Ws + 2 * QCEL + wave * OWEL;
  const int nch = N / QC;
  u32x4 r[QCP];
  auto fetch = [&](int c) {
#pragma unroll
    for (int j = 0; j < QCP; ++j) {
      const int i = tid + 256 * j;
      r[j] = *(const u32x4*)(W + (int64_t)(c * QC + i / (GE / 8)) * GE + (i % (GE / 8)) * 8);
    }
  };
  auto stash = [&](int slot) {
#pragma unroll
    for (int j = 0; j < QCP; ++j) {
      const int i = tid + 256 * j;
      *(u32x4*)(Ws + slot * QCEL + (i / (GE / 8)) * WST + (i % (GE / 8)) * 8) = r[j];
    }
  };
  fetch(0);
  bf16x8 af[2][GE / 32];
#pragma unroll
  for (int tt = 0; tt < 2; ++tt) {
    const int64_t m = min(m0 + tt * 16 + fr, (int64_t)M - 1);
    const TA* xr = A + m * GE + fg * 8;
    f32x4 lo[GE / 32], hi[GE / 32];
#pragma unroll
    for (int ks = 0; ks < GE / 32; ++ks) {
      if constexpr (std::is_same_v<TA, _Float16>) {  // the fp16 mode's MGM tokens
        const f16x8 v = *(const f16x8*)(xr + ks * 32);
#pragma unroll
        for (int i = 0; i < 4; ++i) lo[ks][i] = (float)v[i], hi[ks][i] = (float)v[4 + i];
      } else if constexpr (sizeof(TA) == 2) {
        const bf16x8 v = *(const bf16x8*)(xr + ks * 32);
#pragma unroll
        for (int i = 0; i < 4; ++i) lo[ks][i] = (float)v[i], hi[ks][i] = (float)v[4 + i];
      } else {
        lo[ks] = *(const f32x4*)(xr + ks * 32);
        hi[ks] = *(const f32x4*)(xr + ks * 32 + 4);
      }
    }
    float mean = 0.f, inv = 1.f;
    if (do_ln) {  // the row's 192 features are spread over lanes fr + 16 fg (48 each)
      float sm = 0.f;
#pragma unroll
      for (int ks = 0; ks < GE / 32; ++ks)
#pragma unroll
        for (int i = 0; i < 4; ++i) sm += lo[ks][i] + hi[ks][i];
      mean = sum_rows4(sm) * (1.0f / GE);
      float q = 0.f;
#pragma unroll
      for (int ks = 0; ks < GE / 32; ++ks)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float a = lo[ks][i] - mean, b = hi[ks][i] - mean;
          q += a * a + b * b;
        }
      inv = 1.0f / sqrtf(sum_rows4(q) * (1.0f / GE) + eps);
    }
#pragma unroll
    for (int ks = 0; ks < GE / 32; ++ks) {
      bf16x8 v;
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = (bf16)((lo[ks][i] - mean) * inv), v[4 + i] = (bf16)((hi[ks][i] - mean) * inv);
      af[tt][ks] = v;
    }
  }
  stash(0);
  if (nch > 1) fetch(1);
  __syncthreads();
  for (int c = 0; c < nch; ++c) {
    if (c + 1 < nch) stash((c + 1) & 1);
    if (c + 2 < nch) fetch(c + 2);
    const uint16_t* Wc = Ws + (c & 1) * QCEL;
    f32x4 acc[QC / 16][2];
#pragma unroll
    for (int f = 0; f < QC / 16; ++f) acc[f][0] = acc[f][1] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (vt_from >= 0 && c * QC >= vt_from) {  // block-uniform
      chunk_mma<false>(Wc, af, fr, fg, acc);
      // C: lane = feature 16f + fr, rows 16tt + 4fg + i  ->  Os[feature][row] (+ bias)
#pragma unroll
      for (int f = 0; f < QC / 16; ++f) {
        const float bv = bias[c * QC + f * 16 + fr];
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) {
          bf16x4 o;
#pragma unroll
          for (int i = 0; i < 4; ++i) o[i] = (bf16)(acc[f][tt][i] + bv);
          *(bf16x4*)(Os + (f * 16 + fr) * OVST + tt * 16 + fg * 4) = o;
        }
      }
      if (m0 < M) {  // the wave's 32 rows are keys j0 .. j0 + 31 of group g0 (Mk % 32 == 0, M % Mk == 0)
        const int64_t g0 = m0 / Mk;
        const int j0 = (int)(m0 - g0 * Mk), nv = N - vt_from;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int feat = 16 * i + (lane >> 2), rr = (lane & 3) * 8;
          const u32x4 v = *(const u32x4*)(Os + feat * OVST + rr);
          *(u32x4*)(CT + (g0 * nv + c * QC - vt_from + feat) * Mk + j0 + rr) = v;
        }
      }
      __syncthreads();
      continue;
    }
    chunk_mma<true>(Wc, af, fr, fg, acc);
    // C^T: lane = row 16tt + fr, features 16f + 4fg + i  ->  Os[row][feature] (+ bias)
#pragma unroll
    for (int f = 0; f < QC / 16; ++f) {
      const f32x4 bv = *(const f32x4*)(bias + c * QC + f * 16 + fg * 4);
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) {
        bf16x4 o;
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = (bf16)(acc[f][tt][i] + bv[i]);
        *(bf16x4*)(Os + (tt * 16 + fr) * OQST + f * 16 + fg * 4) = o;
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {  // 32 rows x 8 chunks of 16 B
      const int row = 8 * i + (lane >> 3), cc = lane & 7;
      const u32x4 v = *(const u32x4*)(Os + row * OQST + cc * 8);
      if (m0 + row < M) *(u32x4*)(C + (m0 + row) * ldc + c * QC + cc * 8) = v;  // (C: bf16 elements)
    }
    __syncthreads();
  }
}

template <bool F16>
__global__ __launch_bounds__(256, 2) void rowgemm_resln_kernel(const RgArgs p) {
  typedef typename Op16<F16>::x8 X8;
  __shared__ __attribute__((aligned(16))) uint16_t Ws[GE * WST];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const int64_t m0 = (int64_t)blockIdx.x * GROWS + wave * 32;
  stage_panel((const uint16_t*)p.W, 0, Ws, tid);
  X8 af[2][GE / 32];
  load_rows<false>(p, m0, fr, fg, af);
  __syncthreads();
  f32x4 y[GE / 16][2];
  panel_mma<true>(Ws, af, fr, fg, y);
  // Y^T: lane = row, rows of tile f = features 16f + 4fg + i (F16: f16_row_perm-ordered W rows, features
  // 32(f>>1) + 8fg + 4(f&1) + i -- 16-B runs of the fp16 row)
#pragma unroll
  for (int tt = 0; tt < 2; ++tt) {
    const int64_t m = m0 + tt * 16 + fr;
    const bool valid = m < p.M;
    float* xr = (float*)p.X + (valid ? m : (int64_t)p.M - 1) * GE + fg * 4;
    f16* hr = (f16*)p.X + (valid ? m : (int64_t)p.M - 1) * GE + fg * 8;
    float s = 0.f;
#pragma unroll
    for (int f = 0; f < GE / 16; ++f) {
      f32x4 xv;
      if constexpr (F16) {
        const f16x8 h8 = *(const f16x8*)(hr + (f >> 1) * 32);
#pragma unroll
        for (int i = 0; i < 4; ++i) xv[i] = (float)h8[4 * (f & 1) + i];
      } else {
        xv = *(const f32x4*)(xr + f * 16);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        y[f][tt][i] += xv[i];
        s += y[f][tt][i];
      }
    }
    s = sum_rows4(s);
    const float mean = s * (1.0f / GE);
    float q = 0.f;
#pragma unroll
    for (int f = 0; f < GE / 16; ++f)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float dl = y[f][tt][i] - mean;
        q += dl * dl;
      }
    q = sum_rows4(q);
    const float inv = 1.0f / sqrtf(q * (1.0f / GE) + p.eps);
    if (valid) {
      if constexpr (F16) {
#pragma unroll
        for (int k = 0; k < GE / 32; ++k) {
          f16x8 ov;
#pragma unroll
          for (int i = 0; i < 4; ++i)
            ov[i] = (f16)((y[2 * k][tt][i] - mean) * inv), ov[4 + i] = (f16)((y[2 * k + 1][tt][i] - mean) * inv);
          *(f16x8*)(hr + 32 * k) = ov;
        }
      } else {
#pragma unroll
        for (int f = 0; f < GE / 16; ++f) {
          f32x4 ov;
#pragma unroll
          for (int i = 0; i < 4; ++i) ov[i] = (y[f][tt][i] - mean) * inv;
          *(f32x4*)(xr + f * 16) = ov;
        }
      }
    }
  }
}

}  // namespace

namespace {
// one row set of the QKV projection: args, row tiles per column and block count (0 blocks: M == 0)
hipError_t qkv_rowset(const void* X, int64_t a_rdiv, int64_t a_rmul, int64_t a_rmul2, int64_t a_roff, const void* W,
                      int M, int N, void* q, void* k, void* vt, int S, int Npad, int H, RgArgs& a, int& tiles,
                      int64_t& nblk) {
  a = RgArgs{};
  tiles = 1, nblk = 0;
  if (M <= 0) return hipSuccess;
  if ((N != GE && N != 3 * GE) || H * 32 != GE) return hipErrorInvalidValue;
  a.A = X, a.a_rdiv = a_rdiv, a.a_rmul = a_rmul, a.a_rmul2 = a_rmul2, a.a_roff = a_roff;
  a.W = W, a.M = M, a.N = N;
  a.q = q, a.k = k, a.vt = (bf16*)vt, a.S = S, a.Npad = Npad, a.H = H;
  // blocks tile each column b separately: nb = M / a_rdiv columns of a_rdiv rows
  if (a_rdiv <= 0 || M % a_rdiv != 0) return hipErrorInvalidValue;
  if (N == 3 * GE && (a_roff % 8 != 0 || a_roff + a_rdiv > Npad)) return hipErrorInvalidValue;  // 16-B V^T stores
  tiles = (int)((a_rdiv + GROWS - 1) / GROWS);
  nblk = (int64_t)tiles * (M / a_rdiv);
  return hipSuccess;
}
}  // namespace

hipError_t launch_rowgemm_qkv(const void* X, int64_t a_rdiv, int64_t a_rmul, int64_t a_rmul2, int64_t a_roff,
                              const void* W, int M, int N, void* q, void* k, void* vt, int S, int Npad, int H,
                              hipStream_t st, bool f16, bool qk_bf16) {
  RgArgs a;
  int tiles;
  int64_t nblk;
  hipError_t e = qkv_rowset(X, a_rdiv, a_rmul, a_rmul2, a_roff, W, M, N, q, k, vt, S, Npad, H, a, tiles, nblk);
  if (e != hipSuccess || nblk == 0) return e;
  const dim3 g((unsigned)nblk);
  if (f16 && qk_bf16) hipLaunchKernelGGL((rowgemm_qkv2_kernel<true, true>), g, dim3(256), 0, st, a, tiles, a, tiles, (int)nblk);
  else if (f16) hipLaunchKernelGGL((rowgemm_qkv2_kernel<true, false>), g, dim3(256), 0, st, a, tiles, a, tiles, (int)nblk);
  else hipLaunchKernelGGL((rowgemm_qkv2_kernel<false, false>), g, dim3(256), 0, st, a, tiles, a, tiles, (int)nblk);
  return hipGetLastError();
}

hipError_t launch_rowgemm_qkv_pair(const void* X, int64_t rdiv1, int64_t roff1, const void* W1, int M1, int N1,
                                   int64_t rdiv2, int64_t roff2, const void* W2, int M2, int N2, int64_t a_rmul,
                                   void* q, void* k, void* vt, int S, int Npad, int H, hipStream_t st, bool f16,
                                   bool qk_bf16) {
  RgArgs a1, a2;
  int t1, t2;
  int64_t n1, n2;
  hipError_t e = qkv_rowset(X, rdiv1, a_rmul, 1, roff1, W1, M1, N1, q, k, vt, S, Npad, H, a1, t1, n1);
  if (e != hipSuccess) return e;
  e = qkv_rowset(X, rdiv2, a_rmul, 1, roff2, W2, M2, N2, q, k, vt, S, Npad, H, a2, t2, n2);
  if (e != hipSuccess) return e;
  if (n1 + n2 == 0) return hipSuccess;
  if (n1 == 0) a1 = a2, t1 = t2;  // blocks index the second set only
  const dim3 g((unsigned)(n1 + n2));
  if (f16 && qk_bf16) hipLaunchKernelGGL((rowgemm_qkv2_kernel<true, true>), g, dim3(256), 0, st, a1, t1, a2, t2, (int)n1);
  else if (f16) hipLaunchKernelGGL((rowgemm_qkv2_kernel<true, false>), g, dim3(256), 0, st, a1, t1, a2, t2, (int)n1);
  else hipLaunchKernelGGL((rowgemm_qkv2_kernel<false, false>), g, dim3(256), 0, st, a1, t1, a2, t2, (int)n1);
  return hipGetLastError();
}

hipError_t launch_rowgemm_resln(const void* O, const void* W, int64_t M, void* X, float eps, hipStream_t st, bool f16) {
  if (M <= 0) return hipSuccess;
  RgArgs a{};
  a.A = O, a.a_rdiv = 1, a.a_rmul = 1, a.a_rmul2 = 0, a.a_roff = 0;
  a.W = W, a.M = (int)M, a.N = GE, a.X = X, a.eps = eps;
  const dim3 grid((unsigned)((M + GROWS - 1) / GROWS));
  if (f16) hipLaunchKernelGGL(rowgemm_resln_kernel<true>, grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL(rowgemm_resln_kernel<false>, grid, dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_rowgemm_ln_store(const void* A, bool a_bf16, const void* W, const float* bias, void* C, int64_t M,
                                   int N, float eps, bool ln, hipStream_t st, void* CT, int vt_from, int Mk,
                                   bool a_f16) {
  if (M <= 0) return hipSuccess;
  if (N % QC != 0 || N <= 0 || M > INT32_MAX) return hipErrorInvalidValue;
  if (CT && (vt_from < 0 || vt_from % QC != 0 || vt_from >= N || Mk <= 0 || Mk % 32 != 0 || M % Mk != 0))
    return hipErrorInvalidValue;
  const int ldc = CT ? vt_from : N;
  const dim3 grid((unsigned)((M + GROWS - 1) / GROWS));
  if (a_f16)
    hipLaunchKernelGGL((rowgemm_ln_store_kernel<_Float16>), grid, dim3(256), 0, st, (const _Float16*)A, (const bf16*)W,
                       bias, (bf16*)C, (int)M, N, eps, ln ? 1 : 0, ldc, (bf16*)CT, CT ? vt_from : -1, CT ? Mk : 1);
  else if (a_bf16)
    hipLaunchKernelGGL((rowgemm_ln_store_kernel<bf16>), grid, dim3(256), 0, st, (const bf16*)A, (const bf16*)W, bias,
                       (bf16*)C, (int)M, N, eps, ln ? 1 : 0, ldc, (bf16*)CT, CT ? vt_from : -1, CT ? Mk : 1);
  else
    hipLaunchKernelGGL((rowgemm_ln_store_kernel<float>), grid, dim3(256), 0, st, (const float*)A, (const bf16*)W, bias,
                       (bf16*)C, (int)M, N, eps, ln ? 1 : 0, ldc, (bf16*)CT, CT ? vt_from : -1, CT ? Mk : 1);
  return hipGetLastError();
}

}  // namespace mmpfn
