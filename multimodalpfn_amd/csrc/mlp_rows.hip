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
// Software pipeline over hidden chunks c: GELU(H(c)) on the VALU beside the MFMAs of H(c+1), then
// Y^T += W2c . GELU(H(c)); one barrier per chunk.  Only the weights move through LDS: a 128-row block
// (4 waves) shares each chunk, delivered by LDS-DMA into three-slot W1 / W2 rings (72 KB per block,
// two blocks per CU) two chunks ahead of use, unpadded and XOR-swizzled (see the ring comment below).
// Measured against register staging into two padded slots (in-step launch, rocprofv3): 168-171 ->
// 162-163 us per two-member launch; a DMA ring whose peeled tail chunks spilled 130 VGPRs ran 197 us.
//
// F16 (PREC_F16): X and O are fp16 and every operand is fp16.  The output rows (W2, and Wout of the fused
// prologue) are stored in f16_row_perm order (weight_pack.h), so Y^T tile f row 4g+i is feature
// 32(f>>1) + 8g + 4(f&1) + i: a lane's 48 features are six 16-B runs of the fp16 row (one load / store
// each), and the X^T fragments built from Y^T are in natural feature order (W1 unpermuted).
#include <type_traits>

#include "common.h"
#include "kernels.h"

namespace mmpfn {

namespace {

constexpr int RE = 192;                    // model width
constexpr int RHC = 32;                    // hidden chunk
constexpr int SLOT_B = RHC * RE * 2;       // one W1 or W2 chunk image: 12 KB
constexpr int NSLOT = 3;                   // ring depth per matrix
constexpr int W2RING = NSLOT * SLOT_B;     // byte offset of the W2 ring
constexpr int LDS_B = 2 * NSLOT * SLOT_B;  // 72 KB per block: two blocks per CU
constexpr int MP = SLOT_B / 1024 / 4;      // 1-KB DMA pieces per wave, matrix and chunk (3)
typedef __attribute__((ext_vector_type(2))) float float2_t;

// "m0" in the clobber list: clang keeps m0 reserved and ignores the entry (-Winline-asm; the ISA is identical with
// and without it), and every m0 use the compiler emits itself is preceded by its own write -- test_codegen checks
// that no m0 read other than these DMA issues exists in the kernels
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void mlp_dma16(uint32_t voff, const void* sbase, unsigned lds_dst) {
  // m0 = the wave's LDS destination; lane i's 16 B (sbase + voff) land at m0 + 16 i
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sbase), "s"(lds_dst)
               : "memory", "m0");
}
#pragma clang diagnostic pop

template <typename F, int... I>
__device__ __forceinline__ void static_for_(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {  // f(integral_constant<int, 0>) .. f(<N - 1>)
  static_for_(f, std::make_integer_sequence<int, N>{});
}

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma16(f16x8 a, f16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// TT = 16-row tiles per wave: 2 (32 rows, two waves per SIMD, accumulators in VGPRs) or 4 (64 rows,
// one wave per SIMD with the 192 x 64 Y^T accumulator in AGPRs -- half the LDS weight reads per row,
// but measured 15% slower: one wave cannot hide the LDS / GELU latency the second wave covers)
// NW = waves per block: 4 (two blocks per CU, each DMA-filling its own rings) or 8 (one block per CU:
// each weight byte crosses into LDS once per CU; waves 0-3 fill the W1 ring, 4-7 the W2 ring)
// CAP (with RES, bf16): the CrossAttentionPooler's tail (transformer.py:85-86) on its pooled tokens:
//   o2 = O Wout^T + bo;  X <- LayerNorm(o2) g + b + (GELU(o2 W1^T + b0) W2^T + b3)
// (the prologue's residual is the bias, its LayerNorm moves to the end beside the FFN, exact-erf GELU);
// the vectors [bo | b0 | g | b + b3] sit in LDS beside the rings (capb, CAPL floats).
constexpr int CAPL = 5 * RE;  // bo, b0 (2 RE), g, b + b3

#ifdef MMPFN_STAMPS_ALL  // every wave of the grid: HW_ID, XCC_ID and MR_NST s_memtime stamps (diagnostics only;
// tools/mlp_stamps_all.py): 0 start, 1 O / X / Wout half 0 landed, 2 out-projection half 0, 3 half 1, 4 LayerNorm and
// W1(0) landed, 5 H(0), 6 + c after chunk c (c < 24), MR_NST - 1 after the stores
constexpr int MR_NST = 32, MR_MAXB = 4096;
__device__ unsigned long long g_mr_all[MR_MAXB * 8 * (MR_NST + 2)];
#define MR_STAMP(k)                                                                                     \
  do {                                                                                                  \
    if (!CAP && lane == 0 && blockIdx.x < MR_MAXB && (k) < MR_NST)                                      \
      g_mr_all[((size_t)blockIdx.x * NW + wave) * (MR_NST + 2) + 2 + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define MR_STAMP(k) \
  do {              \
  } while (0)
#endif
template <int TT, bool RES, int NW, bool F16, bool CAP = false>
__global__ __launch_bounds__(64 * NW, NW == 8 ? 1 : (TT == 2 ? 2 : 1)) void mlp_rows_kernel(void* __restrict__ Xv,
                                                                       const void* __restrict__ W1v,
                                                                       const void* __restrict__ W2v, int M, int Fh,
                                                                       float eps, const void* __restrict__ Ov,
                                                                       const void* __restrict__ Woutv,
                                                                       const float* __restrict__ capb) {
  static_assert(!CAP || (RES && !F16), "the CAP tail runs the bf16 prologue form");
  typedef typename Op16<F16>::t HT;  // operand element
  typedef typename Op16<F16>::x8 X8;
  typedef __attribute__((ext_vector_type(2))) HT HT2;
  float* __restrict__ X = (float*)Xv;  // bf16 mode: the fp32 state
  f16* __restrict__ Xh = (f16*)Xv;     // F16: the fp16 state
  const HT* __restrict__ W1 = (const HT*)W1v;
  const HT* __restrict__ W2p = (const HT*)W2v;
  const HT* __restrict__ O = (const HT*)Ov;
  const HT* __restrict__ Wout = (const HT*)Woutv;
  constexpr int RROWS = NW * 16 * TT;  // rows per block
  __shared__ __attribute__((aligned(1024))) bf16 lds[LDS_B / 2];
  __shared__ __attribute__((aligned(16))) float capl[CAP ? CAPL : 4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  MR_STAMP(0);
#ifdef MMPFN_STAMPS_ALL
  if (!CAP && lane == 0 && blockIdx.x < MR_MAXB) {
    const size_t b0 = ((size_t)blockIdx.x * NW + wave) * (MR_NST + 2);
    g_mr_all[b0] = __builtin_amdgcn_s_getreg(4 | (31 << 11));       // HW_REG_HW_ID
    g_mr_all[b0 + 1] = __builtin_amdgcn_s_getreg(20 | (31 << 11));  // HW_REG_XCC_ID
  }
#endif
  if constexpr (CAP)  // before any LDS-DMA: the compiler's own vmcnt waits cover these loads alone
    for (int i = tid; i < CAPL; i += 64 * NW) capl[i] = capb[i];
  const int wg = wave & 3;                           // the wave's share of a ring fill
  const bool gw1 = NW == 4 || wave < 4, gw2 = NW == 4 || wave >= 4;  // fills W1 / W2 pieces
  const int fr = lane & 15, fg = lane >> 4;
  const int64_t m0 = (int64_t)blockIdx.x * RROWS + wave * 16 * TT;
  const int nchunks = Fh / RHC;

  // Weight rings filled by LDS-DMA (global_load_lds_dwordx4 in inline asm, so the compiler adds no
  // vmcnt(0) before reads of the other slots; the kernel waits for its own pieces explicitly): three
  // W1 slots (chunk c+1 read by this chunk's up-projection, c+2 landing, c+3 in flight) and three W2
  // slots (chunk c read, c+1 landing, c+2 in flight), so every fill has two chunks to arrive.  Images
  // are unpadded with 16-B units XOR-swizzled for conflict-free ds_read_b128 fragment reads:
  //   W1 slot [32 rows][384 B]: unit u of row r at (u ^ ((r >> 1) & 7))
  // (conflict-free for ds_read_b128's four lane groups, MI355X_MICROARCH.md LDS table)
  //   W2 slot [192 rows][64 B]: unit u of row r at (u ^ ((r >> 2) & 2))
  // The DMA writes lane-linearly (lane i of a wave instruction -> 16 i of its 1-KB piece), so each
  // lane fetches the unit that belongs at its position: a per-lane 32-bit offset from a uniform
  // chunk base (saddr form), three pieces per wave and matrix per chunk.
  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) void*)lds;
  uint32_t o1[MP], o2[MP];
#pragma unroll
  for (int j = 0; j < MP; ++j) {
    const int q = (wg * MP + j) * 64 + lane;  // unit index inside a slot image
    const int r1 = q / 24, u1 = (q % 24) ^ ((r1 >> 1) & 7);
    o1[j] = (uint32_t)(r1 * RE + u1 * 8) * 2;
    const int r2 = q >> 2, u2 = (q & 3) ^ ((r2 >> 2) & 2);
    o2[j] = (uint32_t)(r2 * Fh + u2 * 8) * 2;
  }
  auto dma_w1 = [&](int c, int slot) {  // W1 rows c*32 .. +31
    if (!gw1) return;
    const HT* base = W1 + (int64_t)c * RHC * RE;
#pragma unroll
    for (int j = 0; j < MP; ++j)
      mlp_dma16(o1[j], base, __builtin_amdgcn_readfirstlane(lds0 + slot * SLOT_B + (wg * MP + j) * 1024));
  };
  auto dma_w2 = [&](int c, int slot) {  // W2 columns c*32 .. +31 (permuted), all 192 rows
    if (!gw2) return;
    const HT* base = W2p + c * RHC;
#pragma unroll
    for (int j = 0; j < MP; ++j)
      mlp_dma16(o2[j], base,
                __builtin_amdgcn_readfirstlane(lds0 + W2RING + slot * SLOT_B + (wg * MP + j) * 1024));
  };
  // fragment read offsets (bytes inside a slot): W1 row 16 ht + fr, unit 4 ks + fg; W2 row 16 o + fr, unit fg
  const int s1 = (fr >> 1) & 7;
  const uint32_t f1e = fr * 384 + ((fg ^ s1) << 4), f1o = fr * 384 + (((4 + fg) ^ s1) << 4);
  const uint32_t f2 = W2RING + fr * 64 + ((fg ^ ((fr >> 2) & 2)) << 4);
  const unsigned char* ldsb = (const unsigned char*)lds;
  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  using S2 = std::integral_constant<int, 2>;

  // ---- the wave's rows as B fragments in the Y^T lane layout: lane (row 16tt + fr, group fg)
  //      holds features 16f + 4fg + i; K position 32ks + 8fg + j <-> feature of tile f = 2ks + j/4
  X8 af[TT][RE / 32];
  f32x4 y[RE / 16][TT];
  auto to_af = [&](int tt) {
#pragma unroll
    for (int ks = 0; ks < RE / 32; ++ks) {
      X8 b;
#pragma unroll
      for (int i = 0; i < 4; ++i) b[i] = (HT)y[2 * ks][tt][i], b[4 + i] = (HT)y[2 * ks + 1][tt][i];
      af[tt][ks] = b;
    }
  };
  auto load_x = [&]() {  // y <- the residual rows X, in the Y^T accumulator layout
#pragma unroll
    for (int tt = 0; tt < TT; ++tt) {
      const int64_t m = min(m0 + tt * 16 + fr, (int64_t)M - 1);
      if constexpr (F16) {  // features 32k + 8fg .. +7 = tiles 2k, 2k+1 (f16_row_perm layout)
        const f16* xr = Xh + m * RE + fg * 8;
#pragma unroll
        for (int k = 0; k < RE / 32; ++k) {
          const f16x8 h = *(const f16x8*)(xr + 32 * k);
#pragma unroll
          for (int i = 0; i < 4; ++i) y[2 * k][tt][i] = (float)h[i], y[2 * k + 1][tt][i] = (float)h[4 + i];
        }
      } else {
        const float* xr = X + m * RE + fg * 4;
#pragma unroll
        for (int f = 0; f < RE / 16; ++f) y[f][tt] = *(const f32x4*)(xr + f * 16);
      }
    }
  };
  auto wait_vm = [](auto nc) {  // s_waitcnt vmcnt(N): all but this thread's N newest memory ops landed
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(decltype(nc)::value) : "memory");
  };
  using std::integral_constant;
  // Ring fill order and waits assume three or more chunks (Fh >= 96); fewer drain everything.
  const bool deep = nchunks >= 3;
  if constexpr (RES) {
    // X <- LayerNorm(X + O . Wout^T): the accumulators start from the residual X, so the out-projection
    // MFMAs add onto it.  Wout [192 out][192 in] arrives by LDS-DMA in two 96-row halves, swizzled like
    // the W1 slots, half 0 over the W1 ring and half 1 over the W2 ring, both at kernel start (under
    // the O / X loads); the W1 ring refills during half 1's MFMAs, the W2 ring during the LayerNorm.
    {
      // piece j of this wave: unit q = (wave * 9 + j) * 64 + lane of a half image: row q / 24, unit
      // (q % 24) ^ ((row >> 1) & 7)
      uint32_t ow[9];
#pragma unroll
      for (int j = 0; j < 9; ++j) {
        const int q = (wg * 9 + j) * 64 + lane, r = q / 24, u = (q % 24) ^ ((r >> 1) & 7);
        ow[j] = (uint32_t)(r * RE + u * 8) * 2;
      }
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        if (hf == 1 && !CAP) load_x();  // (program order: half 0, O, X, half 1 -- see the waits below)
        if (NW == 4 || (wave >> 2) == hf)  // NW 8: waves 0-3 half 0, 4-7 half 1
#pragma unroll
          for (int j = 0; j < 9; ++j)
            mlp_dma16(ow[j], Wout + hf * 96 * RE,
                      __builtin_amdgcn_readfirstlane(lds0 + hf * 3 * SLOT_B + (wg * 9 + j) * 1024));
        if (hf == 0) {
          X8 ao[TT][RE / 32];
#pragma unroll
          for (int tt = 0; tt < TT; ++tt) {
            const int64_t m = min(m0 + tt * 16 + fr, (int64_t)M - 1);
#pragma unroll
            for (int ks = 0; ks < RE / 32; ++ks) ao[tt][ks] = *(const X8*)(O + m * RE + ks * 32 + fg * 8);
          }
#pragma unroll
          for (int tt = 0; tt < TT; ++tt)
#pragma unroll
            for (int ks = 0; ks < RE / 32; ++ks) af[tt][ks] = ao[tt][ks];  // O parked in af until the LN
        }
      }
    }
    auto outproj = [&](auto hc) {  // y[6 hf .. 6 hf + 5] += Wout half hf . O^T
      constexpr int HF = decltype(hc)::value;
#pragma unroll
      for (int ks = 0; ks < RE / 32; ++ks)
#pragma unroll
        for (int fl = 0; fl < 6; ++fl) {
          const X8 w = *(const X8*)(ldsb + HF * 3 * SLOT_B + fl * 16 * 384 + (ks >> 1) * 128 +
                                    ((ks & 1) ? f1o : f1e));
#pragma unroll
          for (int tt = 0; tt < TT; ++tt) y[6 * HF + fl][tt] = mfma16(w, af[tt][ks], y[6 * HF + fl][tt]);
        }
    };
    wait_vm(integral_constant<int, 9>{});  // half 0 (and O, X) landed; half 1 may fly
    __syncthreads();
    MR_STAMP(1);
    if constexpr (CAP)  // the out-projection accumulates onto its bias
#pragma unroll
      for (int tt = 0; tt < TT; ++tt)
#pragma unroll
        for (int f = 0; f < RE / 16; ++f) y[f][tt] = *(const f32x4*)(capl + f * 16 + fg * 4);
    outproj(integral_constant<int, 0>{});
    __syncthreads();  // every wave is done with half 0: the W1 ring is free
    MR_STAMP(2);
    dma_w1(0, 0);
    if (nchunks > 1) dma_w1(1, 1);
    if (deep) dma_w1(2, 2);
    // half 1 landed, the W1 fills may fly (NW 8: waves 0-3 hold no half-1 pieces, 4-7 no W1 fills)
    if (deep && gw1) wait_vm(integral_constant<int, 3 * MP>{});
    else wait_vm(integral_constant<int, 0>{});
    __syncthreads();
    outproj(integral_constant<int, 1>{});
    __syncthreads();  // the W2 ring is free
    MR_STAMP(3);
    dma_w2(0, 0);
    if (nchunks > 1) dma_w2(1, 1);
    // residual (already in y) + LayerNorm (layer.py:437-455), packed as the MLP's A^T fragments
    float mu[TT], iv[TT];
#pragma unroll
    for (int tt = 0; tt < TT; ++tt) {
      float sm = 0.f;
#pragma unroll
      for (int f = 0; f < RE / 16; ++f)
#pragma unroll
        for (int i = 0; i < 4; ++i) sm += y[f][tt][i];
      const float mean = sum_rows4(sm) * (1.0f / RE);
      float q = 0.f;
#pragma unroll
      for (int f = 0; f < RE / 16; ++f)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float dl = y[f][tt][i] - mean;
          q += dl * dl;
        }
      mu[tt] = mean, iv[tt] = 1.0f / sqrtf(sum_rows4(q) * (1.0f / RE) + eps);
      if constexpr (CAP) {
        to_af(tt);  // the FFN reads o2 itself
      } else {
#pragma unroll
        for (int f = 0; f < RE / 16; ++f)
#pragma unroll
          for (int i = 0; i < 4; ++i) y[f][tt][i] = (y[f][tt][i] - mean) * iv[tt];
        to_af(tt);
      }
    }
    if constexpr (CAP) {  // y restarts as out_norm(o2) + b3: one tile's g / (b + b3) live at a time
#pragma unroll
      for (int f = 0; f < RE / 16; ++f) {
        asm volatile("" ::: "memory");  // (g / b loads hoisted above the LayerNorm spilled ~110 VGPRs)
        const int e = f * 16 + fg * 4;
        const f32x4 g = *(const f32x4*)(capl + 3 * RE + e), bb = *(const f32x4*)(capl + 4 * RE + e);
#pragma unroll
        for (int tt = 0; tt < TT; ++tt)
#pragma unroll
          for (int i = 0; i < 4; ++i) y[f][tt][i] = fmaf((y[f][tt][i] - mu[tt]) * iv[tt], g[i], bb[i]);
      }
    }
    // before H(0): W1(0) landed (newer: W1(1), W1(2), W2(0), W2(1); NW 8: each group its own two)
    if (deep) wait_vm(integral_constant<int, (NW == 8 ? 2 : 4) * MP>{});
    else wait_vm(integral_constant<int, 0>{});
  } else {
    dma_w1(0, 0);
    if (nchunks > 1) dma_w1(1, 1);
    load_x();
#pragma unroll
    for (int tt = 0; tt < TT; ++tt) to_af(tt);
    dma_w2(0, 0);
    if (deep) dma_w1(2, 2);
    if (nchunks > 1) dma_w2(1, 1);
    // before H(0): W1(0) landed (newer: W1(1), W2(0), W1(2), W2(1); NW 8: W1(1), X, W1(2))
    if (deep) wait_vm(integral_constant<int, (NW == 8 ? 2 : 4) * MP>{});
    else wait_vm(integral_constant<int, 0>{});
  }
  __syncthreads();
  MR_STAMP(4);

  // GELU of one adjacent pair q (0 .. 4 TT - 1: tile tt, half ht, elements 2 (q & 1) + 0, 1) of a chunk's
  // H^T accumulators, packed into its bf16 B fragment for the down-projection
#ifndef MLP_GELU16
#define MLP_GELU16 3  // 3: gelu_tanh_h2x2_f32, 2: gelu_tanh_h2x2, 1: one pair per gelu_tanh_h2, 0: fp32 tanh form
#endif
  auto gelu_pair = [&](auto qc, const f32x4 (&hs)[2][TT], X8 (&hb)[TT], int c) {
    constexpr int q = decltype(qc)::value, tt = q >> 2, ht = (q >> 1) & 1, i = 2 * (q & 1);
    HT2 pr;
    if constexpr (CAP) {  // hidden bias b0 (hidden c*32 + 16 ht + 4 fg + i of the H^T tile), exact GELU
      const float2_t bb = *(const float2_t*)(capl + RE + c * RHC + 16 * ht + 4 * fg + i);
      pr = __builtin_convertvector((float2_t){gelu_erf(hs[ht][tt][i] + bb[0]), gelu_erf(hs[ht][tt][i + 1] + bb[1])},
                                   HT2);
    } else if constexpr (F16 && MLP_GELU16 == 3) {  // fp16 mode: pairs q, q + 1 from the fp32 accumulators
      if constexpr ((q & 1) == 0) {
        f16x2_t a, b;
        gelu_tanh_h2x2_f32(hs[ht][tt][0], hs[ht][tt][1], hs[ht][tt][2], hs[ht][tt][3], a, b);
        hb[tt][4 * ht + 0] = a[0], hb[tt][4 * ht + 1] = a[1];
        hb[tt][4 * ht + 2] = b[0], hb[tt][4 * ht + 3] = b[1];
      }
      return;
    } else if constexpr (F16 && MLP_GELU16 == 2) {  // fp16 mode: pairs q, q + 1 (one tile row's four values) at once
      if constexpr ((q & 1) == 0) {
        f16x2_t a = __builtin_convertvector((float2_t){hs[ht][tt][0], hs[ht][tt][1]}, f16x2_t);
        f16x2_t b = __builtin_convertvector((float2_t){hs[ht][tt][2], hs[ht][tt][3]}, f16x2_t);
        gelu_tanh_h2x2(a, b);
        hb[tt][4 * ht + 0] = a[0], hb[tt][4 * ht + 1] = a[1];
        hb[tt][4 * ht + 2] = b[0], hb[tt][4 * ht + 3] = b[1];
      }
      return;
    } else if constexpr (F16 && MLP_GELU16) {  // fp16 mode: the pair's GELU in packed fp16 arithmetic
      pr = gelu_tanh_h2(__builtin_convertvector((float2_t){hs[ht][tt][i], hs[ht][tt][i + 1]}, HT2));
    } else {
      pr = __builtin_convertvector((float2_t){gelu_tanh_fast(hs[ht][tt][i]), gelu_tanh_fast(hs[ht][tt][i + 1])}, HT2);
    }
    hb[tt][4 * ht + i] = pr[0];
    hb[tt][4 * ht + i + 1] = pr[1];
  };
  // H^T [32 hidden][16 TT rows] = W1c . A^T  (W1c in W1 slot SL); with G, the previous chunk's GELU
  // (hs -> hb) rides in the k-steps' MFMA shadows (pairs 0..4TT-1 spread over the RE/32 k-steps)
  auto hmma = [&](auto slc, f32x4 (&h)[2][TT], auto gc, const f32x4 (&hs)[2][TT], X8 (&hb)[TT], int c) {
    constexpr bool G = decltype(gc)::value;
    constexpr int SL = decltype(slc)::value;
    auto w1frag = [&](int ht, int ks) {
      return *(const X8*)(ldsb + SL * SLOT_B + ht * 16 * 384 + (ks >> 1) * 128 + ((ks & 1) ? f1o : f1e));
    };
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int tt = 0; tt < TT; ++tt) h[i][tt] = f32x4{0.f, 0.f, 0.f, 0.f};
#ifndef MLP_PU
#define MLP_PU 2
#endif
    constexpr int PU = MLP_PU;  // k-steps of W1 fragments in flight ahead of their MFMAs
    X8 wa[PU][2];
#pragma unroll
    for (int i = 0; i < PU; ++i)
#pragma unroll
      for (int ht = 0; ht < 2; ++ht) wa[i][ht] = w1frag(ht, i);
#pragma unroll
    for (int ks = 0; ks < RE / 32; ++ks) {
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int ht = 0; ht < 2; ++ht)
#pragma unroll
        for (int tt = 0; tt < TT; ++tt) h[ht][tt] = mfma16(wa[ks % PU][ht], af[tt][ks], h[ht][tt]);
      if (ks + PU < RE / 32)
#pragma unroll
        for (int ht = 0; ht < 2; ++ht) wa[ks % PU][ht] = w1frag(ht, ks + PU);
      if constexpr (G) {  // pairs [ks * NPQ / NKS, (ks + 1) * NPQ / NKS)
        constexpr int NPQ = 4 * TT, NKS = RE / 32;
        static_for<NPQ>([&](auto qc) {
          constexpr int q = decltype(qc)::value;
          if (q * NKS / NPQ == ks) gelu_pair(qc, hs, hb, c);
        });
      }
    }
  };
  // y holds the residual (X, or X' after the fused prologue) in fp32: the down-projection MFMAs
  // accumulate onto it, so the residual is never written out and read back
  f32x4 h[2][TT];
  {
    X8 unused[TT];
    hmma(S0{}, h, std::false_type{}, h, unused, 0);
  }
  // before chunk 0: W1(1) and W2(0) landed (only W2(1) may fly); the barrier also keeps chunk 0 from
  // refilling W1 slot 0 (with W1(3)) while a lagging wave still reads W1(0) above
  if (deep) wait_vm(integral_constant<int, MP>{});
  else wait_vm(integral_constant<int, 0>{});
  __syncthreads();
  MR_STAMP(5);

  // one chunk c (PAR = c % 3): reads W1(c+1) from W1 slot (c+1)%3 and W2(c) from W2 slot c%3;
  // refills W1 slot c%3 (W1(c), read in chunk c-1) with W1(c+3) and W2 slot (c+2)%3 (W2(c-1)) with
  // W2(c+2); at its end W1(c+2) and W2(c+1), issued a chunk earlier, must have landed
  auto chunk = [&](int c, auto parc) {
    const bool MORE = c + 1 < nchunks;  // a chunk c+1 exists (wave-uniform)
    constexpr int PAR = decltype(parc)::value;
    [[maybe_unused]] const bool d1 = c + 3 < nchunks, d2 = c + 2 < nchunks;
    // (issuing these six pieces one per k-step of the up-projection below, beside the GELU, measured
    // neutral for fp16 and 1.5 % slower for bf16: profiles/r04/ab_mlp_gelu16_dma_spread.txt)
    if (d1) dma_w1(c + 3, PAR);
    if (d2) dma_w2(c + 2, (PAR + 2) % 3);
    // GELU of chunk c (VALU) inside the up-projection MFMAs of chunk c+1.  No branch on MORE: the last
    // chunk's up-projection reads a slot holding an older chunk (landed, unused result), which costs 1/24
    // of the up-projections and measured 0.7 % faster than the branch (159.9 -> 158.8 us)
    X8 hb[TT];
    {
      f32x4 hn[2][TT];
      hmma(std::integral_constant<int, (PAR + 1) % 3>{}, hn, std::true_type{}, h, hb, c);
#pragma unroll
      for (int ht = 0; ht < 2; ++ht)
#pragma unroll
        for (int tt = 0; tt < TT; ++tt) h[ht][tt] = hn[ht][tt];
    }
    // Y^T [192][32 rows] += W2c(perm) . GELU(H^T)
    {  // W2 fragments 4 tiles ahead of their MFMAs (fenced so the reads stay early; 3-6 measured)
#ifndef MLP_PF
#define MLP_PF 4
#endif
      constexpr int PF = MLP_PF;
      auto w2frag = [&](int o) { return *(const X8*)(ldsb + PAR * SLOT_B + o * 16 * 64 + f2); };
      X8 wb[PF];
#pragma unroll
      for (int i = 0; i < PF; ++i) wb[i] = w2frag(i);
#pragma unroll
      for (int o = 0; o < RE / 16; ++o) {
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int tt = 0; tt < TT; ++tt) y[o][tt] = mfma16(wb[o % PF], hb[tt], y[o][tt]);
        if (o + PF < RE / 16) wb[o % PF] = w2frag(o + PF);
      }
    }
    if (MORE) {
      // this thread's pieces of W1(c+2) and W2(c+1) landed; this chunk's own fills may still fly
      if constexpr (NW == 8) {  // one matrix per wave
        if (gw1 ? d1 : d2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(MP) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      } else {
        if (d1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * MP) : "memory");
        else if (d2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(MP) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __syncthreads();
    }
#ifdef MMPFN_STAMPS_ALL
    if (c < MR_NST - 7) MR_STAMP(6 + c);
#endif
  };
  // unrolled by three so that every ring slot is a compile-time offset (no peeled copies: the last
  // chunk's "no successor" is a uniform branch)
  for (int c = 0; c < nchunks; c += 3) {
    chunk(c, S0{});
    if (c + 1 < nchunks) chunk(c + 1, S1{});
    if (c + 2 < nchunks) chunk(c + 2, S2{});
  }

  // residual + LayerNorm: lane = row, 48 of its 192 features (rows 16o + 4g + i of Y^T)
#pragma unroll
  for (int tt = 0; tt < TT; ++tt) {
    const int64_t m = m0 + tt * 16 + fr;
    const bool valid = m < M;
    float* xr = X + (valid ? m : (int64_t)M - 1) * RE + fg * 4;
    if constexpr (CAP) {  // out_norm(o2) + b3 + FFN: no LayerNorm after the sum
      if (valid)
#pragma unroll
        for (int o = 0; o < RE / 16; ++o) *(f32x4*)(xr + o * 16) = y[o][tt];
      continue;
    }
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
      if constexpr (F16) {
        f16* hr = Xh + m * RE + fg * 8;
#pragma unroll
        for (int k = 0; k < RE / 32; ++k) {
          f16x8 ov;
#pragma unroll
          for (int i = 0; i < 4; ++i)
            ov[i] = (f16)((y[2 * k][tt][i] - mean) * inv), ov[4 + i] = (f16)((y[2 * k + 1][tt][i] - mean) * inv);
          *(f16x8*)(hr + 32 * k) = ov;
        }
      } else {
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
  MR_STAMP(MR_NST - 1);
}

}  // namespace

namespace {
template <bool F16>
hipError_t launch_mr(void* X, const void* W1, const void* W2, int64_t M, int Fh, float eps, hipStream_t st,
                     const void* O, const void* Wout);
}  // namespace

#ifdef MMPFN_STAMPS_ALL
extern "C" int mmpfn_dbg_mlp_stamps_all(unsigned long long* out, int nblocks) {
  const size_t n = (size_t)(nblocks < MR_MAXB ? nblocks : MR_MAXB) * 8 * (MR_NST + 2) * sizeof(unsigned long long);
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_mr_all), n);
}
#endif

hipError_t launch_cap_tail(const void* O, const void* Wout, const void* W1perm, const void* W2perm, const float* vecs,
                           float* out, int64_t M, int E, float eps, hipStream_t st) {
  if (M <= 0) return hipSuccess;
  if (E != RE || !O || !Wout || !W1perm || !W2perm || !vecs || !out) return hipErrorInvalidValue;
  constexpr int RROWS = 16 * 4 * 2;
  hipLaunchKernelGGL((mlp_rows_kernel<2, true, 4, false, true>), dim3((unsigned)((M + RROWS - 1) / RROWS)), dim3(256),
                     0, st, (void*)out, W1perm, W2perm, (int)M, 2 * RE, eps, O, Wout, vecs);
  return hipGetLastError();
}

hipError_t launch_mlp_rows(void* X, const void* W1perm, const void* W2perm, int64_t M, int E, int Fh, float eps,
                           hipStream_t st, const void* O, const void* Wout, bool f16) {
  if (M <= 0) return hipSuccess;
  if (E != RE || Fh % RHC != 0) return hipErrorInvalidValue;
  return f16 ? launch_mr<true>(X, W1perm, W2perm, M, Fh, eps, st, O, Wout)
             : launch_mr<false>(X, W1perm, W2perm, M, Fh, eps, st, O, Wout);
}

namespace {
template <bool F16>
hipError_t launch_mr(void* X, const void* W1perm, const void* W2perm, int64_t M, int Fh, float eps, hipStream_t st,
                     const void* O, const void* Wout) {
#ifndef MLP_TT
#define MLP_TT 2  // 4 measured slower: 202 vs 175 us per two-member launch
#endif
#ifndef MLP_NW
#define MLP_NW 4  // 8 measured slower: 175.3 vs 162.8 us (one block per CU: its waves hit the barriers in step)
#endif
  constexpr int RROWS = 16 * MLP_NW * MLP_TT;
  const dim3 grid((unsigned)((M + RROWS - 1) / RROWS)), block(64 * MLP_NW);
  if (O)
    hipLaunchKernelGGL((mlp_rows_kernel<MLP_TT, true, MLP_NW, F16>), grid, block, 0, st, X, W1perm, W2perm, (int)M,
                       Fh, eps, O, Wout, nullptr);
  else
    hipLaunchKernelGGL((mlp_rows_kernel<MLP_TT, false, MLP_NW, F16>), grid, block, 0, st, X, W1perm, W2perm, (int)M,
                       Fh, eps, nullptr, nullptr, nullptr);
  return hipGetLastError();
}
}  // namespace

}  // namespace mmpfn
