// Internal launch interface of the MMPFN HIP kernels (not part of the C-ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "weight_pack.h"

namespace mmpfn {

// PREC_F32 (parity mode): every large contraction on bf16 MFMA with both operands split into
// bf16 hi + lo planes, x = hi + lo to 2^-17, and the three significant products hi.hi + hi.lo +
// lo.hi accumulated in fp32 (the dropped lo.lo term is 2^-16 relative) -- 3 bf16 MFMAs at 16x the
// fp32-input rate; PREC_F32_MFMA: the same forward on fp32-input MFMA (exact fp32 fma chains)
// PREC_F16: the reference's fp16 autocast -- the inter-kernel state X stored in fp16, every layer
// contraction on fp16 MFMA operands (the item attention's P.V on bf16: its P needs bf16's range), fp32
// accumulation, LayerNorm and softmax statistics (featrow / rowgemm / mlp_rows / attention_pipe F16 forms)
// PREC_*_F8 / PREC_*_F8E5: the 16-bit modes with the sample-axis attention's P.V on block-scaled fp8
// MFMA (V^T e4m3; P e4m3 / e5m2; attention_pipe.hip) -- config E's fp8 path, opt-in
enum Prec : int {
  PREC_F32 = 0,
  PREC_BF16 = 1,
  PREC_F32_MFMA = 2,
  PREC_BF16_F8 = 3,
  PREC_BF16_F8E5 = 4,
  PREC_F16 = 5,
  PREC_F16_F8 = 6,
  PREC_F16_F8E5 = 7
};
// the precision the layer kernels run in, and the fp8 P.V variant (0: none)
inline int base_prec(int p) {
  return p == PREC_BF16_F8 || p == PREC_BF16_F8E5 ? PREC_BF16 : p == PREC_F16_F8 || p == PREC_F16_F8E5 ? PREC_F16 : p;
}
inline int f8_of(int p) {
  return p == PREC_BF16_F8 || p == PREC_F16_F8 ? 1 : p == PREC_BF16_F8E5 || p == PREC_F16_F8E5 ? 2 : 0;
}
inline bool prec_ok(int p) { return p >= PREC_F32 && p <= PREC_F16_F8E5; }
inline bool prec16(int p) { return p == PREC_BF16 || p == PREC_F16; }  // a 16-bit performance mode (base)

enum Epi : int {
  EPI_STORE = 0,      // C[row] = act(acc + bias)
  EPI_ITEM_QKV = 1,   // scatter to attention Q / K / V^T layouts: row m -> (b = m / a_rdiv, pos = a_roff + m % a_rdiv)
                      //   Q [b][h][pos][32] (S rows), K [b][h][pos][32] (Npad rows), V^T [b][h][32][Npad]
  EPI_RES_LN = 3,     // X[row] = LayerNorm(X[row] + acc), N == 192 (no affine)
  EPI_GLU = 4,        // paired tiles: out = a * sigmoid(b) (weights row-interleaved)
  EPI_REMAP = 5,      // grouped: dest row = (m / rdiv2) * rmul2 + z * zmul + m % rdiv2
};

enum Act : int { ACT_NONE = 0, ACT_GELU = 1 };

struct GemmArgs {
  // A: logical row m -> memory row (m / a_rdiv) * a_rmul + (m % a_rdiv) * a_rmul2 + a_roff
  const void* A;
  int64_t lda;
  int64_t a_rdiv, a_rmul, a_rmul2, a_roff;
  int64_t a_zstride;  // elements between groups (blockIdx.z)
  const void* W;      // [N][K] compute dtype, row-major (PREC_F32: the bf16 hi plane)
  int64_t w_zstride;
  int64_t w_lo_off;   // PREC_F32: elements from W to its bf16 lo plane
  const float* bias;  // [N] or null
  int64_t b_zstride;
  int M, N, K;
  int act;
  // plain / remap / glu output
  void* C;
  int64_t ldc;
  int64_t c_zstride;
  int64_t rdiv2, rmul2, zmul;
  // attention scatter
  void* q;  // Q  [B][H][S][d]
  void* k;  // K  [B][H][Npad][d]
  void* v;  // V^T[B][H][d][Npad]
  int S, Npad, T, H;
  // LN epilogue
  float* X;  // residual in / normalised out, ld = 192
  float ln_eps;
};

// Launch C = A . W^T with the given epilogue.  `a_f32` says whether A is stored
// as fp32 (otherwise bf16); `out_f32` likewise for C / scatter targets.
hipError_t launch_gemm(const GemmArgs& a, int prec, int epi, bool a_f32, bool out_f32, int groups,
                       hipStream_t st);

// MGM head bank, bf16 (fp16 with f16: A, W and C fp16): C[M][N/2] = GLU(A[M][K] . W^T + bias) with W rows GLU-interleaved in 16-row
// blocks (capi.cpp); large-tile, XCD-ordered (gemm.hip gemm_glu_big_kernel); N % 256 == 0, K % 64 == 0
// MGM per-head down-projection (bf16, E = 192): C[(r / n_mod) * nheads n_mod + z n_mod + r % n_mod][E] =
// A[r][z K .. z K + K) (row stride lda) . W[z][E][K]^T + bias[z][E]; C fp32 or bf16 (c_bf16); with f16, A and W
// fp16 and C fp32 or fp16 (c_bf16)
hipError_t launch_gemm_remap_big(const void* A, int64_t lda, const void* W, const float* bias, void* C, bool c_bf16,
                                 int M, int K, int nheads, int n_mod, int E, hipStream_t st, bool f16 = false);
hipError_t launch_gemm_glu_big(const void* A, const void* W, const float* bias, void* C, int M, int N, int K,
                               hipStream_t st, bool f16 = false);

// fused MLP sublayer: X <- LN(X + GELU(X W1^T) W2^T), W1 [Fh][E], W2 [E][Fh] in compute dtype
hipError_t launch_mlp_fused(float* X, const void* W1, const void* W2, int64_t M, int E, int Fh, float eps, int prec,
                            hipStream_t st);

// row-resident MLP sublayer (bf16 only, mlp_rows.hip): W1 [Fh][E] bf16, W2 [E][Fh] bf16 in the
// permuted hidden order of pack_mlp2_perm (capi.cpp); Fh % 32 == 0, E == 192
// W1perm: W1 with its K (feature) order permuted to the Y^T lane layout (capi.cpp pack_mlp1_perm);
// O / Wout non-null: X <- LN(X + O Wout^T) first (the item-attention out-projection, fused)
// f16 (PREC_F16): X / O fp16, W1 natural, W2 (pack_mlp2_perm) and Wout with f16_row_perm-ordered rows
hipError_t launch_mlp_rows(void* X, const void* W1perm, const void* W2perm, int64_t M, int E, int Fh, float eps,
                           hipStream_t st, const void* O = nullptr, const void* Wout = nullptr, bool f16 = false);

// row-resident item-attention projections (bf16, K = 192, rowgemm.hip):
//   QKV: X rows (remap (m/rdiv)*rmul + (m%rdiv)*rmul2 + roff) . W^T, W [N][192] (N = 576 or 192),
//        scattered to Q [b][h][pos][32], K [b][h][pos][32] (Npad rows), V^T [b][h][32][Npad],
//        b = m / rdiv, pos = roff + m % rdiv
//   RES_LN: X <- LN(X + O . W^T), O [M][192] bf16, W [192][192] bf16
//   f16 (PREC_F16): X fp16, W fp16, Q / K fp16 (V^T stays bf16); RES_LN: O / X fp16, W rows in
//   f16_row_perm order (weight_pack.h)
hipError_t launch_rowgemm_qkv(const void* X, int64_t a_rdiv, int64_t a_rmul, int64_t a_rmul2, int64_t a_roff,
                              const void* W, int M, int N, void* q, void* k, void* vt, int S, int Npad, int H,
                              hipStream_t st, bool f16 = false, bool qk_bf16 = false);  // qk_bf16: f16 X, bf16 Q / K
// two row sets (train rows: q|k|v, test rows: q) of the same token columns in ONE launch,
// rows m -> memory row (m / rdiv) * a_rmul + m % rdiv + roff of each set
hipError_t launch_rowgemm_qkv_pair(const void* X, int64_t rdiv1, int64_t roff1, const void* W1, int M1, int N1,
                                   int64_t rdiv2, int64_t roff2, const void* W2, int M2, int N2, int64_t a_rmul,
                                   void* q, void* k, void* vt, int S, int Npad, int H, hipStream_t st,
                                   bool f16 = false, bool qk_bf16 = false);
// C = (ln ? LayerNorm(A) : A) . W^T + bias: A fp32, bf16 or fp16 (a_f16) [M][192], W [N][192] bf16, C bf16 [M][N], N % 64 == 0;
// with CT: outputs [vt_from, N) transposed per group of Mk rows into CT [M / Mk][N - vt_from][Mk] (Mk % 32 == 0),
// C then [M][vt_from]
hipError_t launch_rowgemm_ln_store(const void* A, bool a_bf16, const void* W, const float* bias, void* C, int64_t M,
                                   int N, float eps, bool ln, hipStream_t st, void* CT = nullptr, int vt_from = -1,
                                   int Mk = 0, bool a_f16 = false);
hipError_t launch_rowgemm_resln(const void* O, const void* W, int64_t M, void* X, float eps, hipStream_t st,
                                bool f16 = false);

// parity-mode (x3 split-bf16) row-resident projections of width 192 (rowgemm3.hip), fp32 in and out:
// W = the hi plane [N][192] of capi.cpp upsplit, its lo plane at W + w_lo elements.
//   QKV: up to two row sets in one launch (same remap / scatter as launch_rowgemm_qkv, fp32 Q / K / V^T)
//   RES_LN: X <- LN(X + O . W^T), O fp32 [M][192]
struct Proj3Set {
  const float* A;
  int64_t a_rdiv, a_rmul, a_rmul2, a_roff;
  const void* W;
  int64_t w_lo;
  int M, N;  // N = 576 (q | k | v) or 192 (q)
};
hipError_t launch_proj3_qkv(const Proj3Set* sets, int nset, void* q, void* k, void* vt, int S, int Npad, int H,
                            hipStream_t st);
hipError_t launch_proj3_resln(const float* O, const void* W, int64_t w_lo, int64_t M, float* X, float eps,
                              hipStream_t st);

// row-resident attention-between-features sublayer (bf16 only, featrow.hip): one wave per
// table row, T <= 64 tokens; `pack` (capi.cpp pack_feat_rows) = LDS images with 416-B rows:
// per head [96][FEAT_IMG_STRIDE] (Wq rows permuted & scaled by log2(e)/sqrt(32) | Wk rows
// permuted | Wv), then the out-projection [192][FEAT_IMG_STRIDE] with permuted head columns
// (FEAT_IMG_STRIDE, FEAT_PACK_LAYER: weight_pack.h)
// X holds M members [M][T][S][E]; one launch covers the M*S rows
// f16: PREC_F16 -- X fp16, pack the fp16 images with the out-projection rows permuted (pack_feat_rows res_perm)
hipError_t launch_feat_rows(void* X, const void* pack, int S, int T, int M, int E, int H, float eps, hipStream_t st,
                            bool f16 = false);

// fused attention-between-features sublayer (bf16 only): X <- LN(X + MHA_feat(X)) per row,
// wqkv [3*H*32][E] bf16, wout [E][H*32] bf16; rows per block = feat_block_rows(T) (0: unsupported T)
int feat_block_rows(int T);
hipError_t launch_feat_block(float* X, const void* wqkv, const void* wout, int S, int T, int E, int H, float eps,
                             hipStream_t st);

// ---- attention -------------------------------------------------------------------
// generic MFMA attention over a batch (blockIdx.z) of independent sequences:
//   Q  [b][h][pos][32] (row = s0 + q), K [b][kvh][key][32], V^T [b][kvh][32][kpad],
//   O row = b * o_bstride + (s0 + q) * o_qstride, element row*(H*32) + h*32 + d.
struct AttnArgs {
  const void* q;
  const void* k;
  const void* vt;
  void* o;
  int64_t q_bstride, q_hstride, kv_bstride, kv_hstride;
  int kpad;
  int64_t o_bstride, o_qstride;
  int s0, nq, nk, kvh_fixed, H;
};
hipError_t launch_attn(const AttnArgs& a, int batches, int prec, int waves_per_block, hipStream_t st);
// task map + operands of the sample-axis attention kernels (attention.hip, attention_pipe.hip)
struct Attn2Args {
  const __bf16* q;  // [B][H][S][32]
  const __bf16* k;  // [B][H][Npad][32]
  const __bf16* vt; // [B][H][32][Npad]
  __bf16* o;        // row b*S + s, element row*H*32 + h*32 + d
  int S, H, Npad, nk;
  int a0, na;          // own-head query rows
  int b0, nb, kvb;     // shared-KV query rows (all heads) against kv head kvb
  int tasks_per_b, nblocks;
  int tstart[9];       // task prefix per kv head inside one column
  int64_t kv_bstride;  // elements between the K (V^T) blocks of consecutive columns: H*Npad*32, or
                       // Npad*32 for a head-0-only train-KV cache
  int q_prescaled;     // Q already carries log2(e)/sqrt(32) (folded into the engine's bf16 Q weights)
  const unsigned char* vt8;  // f8 != 0: V^T in e4m3, the layout of vt
  int f8;              // P.V on fp8 MFMA: 0 off (bf16), 1 P in e4m3, 2 P in e5m2 (attention_pipe.hip)
  int qk_f16;          // q, k and o hold fp16 (S on f16 MFMA; the fp16 tap); vt stays bf16
  int o_f16;           // PREC_F16's forward: q, k bf16, o fp16 (every MFMA a bf16 one)
};
// software-pipelined bf16 sample-axis attention (attention_pipe.hip); tasks of ATTN_ITEM_QPB queries
constexpr int ATTN_ITEM_QPB = 256;
hipError_t launch_attn_pipe(const Attn2Args& a, hipStream_t st);
// bf16 sample-axis attention of one layer in one launch (attention_pipe.hip, attn_pipe_kernel):
//   own-head rows [a0, a0+na) of every head against that head's K/V, and rows [b0, b0+nb) of
//   every head against K/V head kvb (nb = 0: none); keys [0, nk), Npad % 64 == 0.
//   kv_bstride > 0: K / V^T hold head 0 only, column blocks kv_bstride elements apart (train-KV
//   cache; then na = 0 and kvb = 0)
//   f8 != 0: P.V and the row sums on block-scaled fp8 MFMA with vt8 = V^T in e4m3 (launch_vt_fp8), P in
//   e4m3 (1) or e5m2 (2); vt (bf16) still serves the exact re-run path
hipError_t launch_attn_layer(const void* q, const void* k, const void* vt, void* out, int S, int T, int H, int Npad,
                             int nk, int a0, int na, int b0, int nb, int kvb, hipStream_t st, int64_t kv_bstride = 0,
                             bool q_prescaled = false,  // Q already scaled by log2(e)/sqrt(32)
                             const void* vt8 = nullptr, int f8 = 0, bool qk_f16 = false, bool o_f16 = false);
// bf16 -> e4m3 (saturating) of n elements (n % 8 == 0): the F8 attention's V^T operand
hipError_t launch_vt_fp8(const void* vt, void* vt8, int64_t n, hipStream_t st);
// parity mode (PREC_F32) of launch_attn_layer on fp32 Q / K / V^T (split bf16 three-product MFMAs), fp32 O
int set_x3_cheap_min_keys(int n, int form);  // previous value; mmpfn_set_parity_attention_min_keys
hipError_t launch_attn_item3(const void* q, const void* k, const void* vt, void* out, int S, int T, int H, int Npad,
                             int nk, int a0, int na, int b0, int nb, int kvb, hipStream_t st, int64_t kv_bstride = 0);
// item attention: queries s in [s0, s0+nq), keys [0, nk); kv_head_fixed >= 0 forces that KV head
hipError_t launch_attn_item(const void* q, const void* k, const void* vt, void* out, int S, int T, int H,
                            int Npad, int s0, int nq, int nk, int kv_head_fixed, int prec, hipStream_t st,
                            int64_t kv_bstride = 0);

// ---- encoders / decoder ------------------------------------------------------------
struct SlotParams {  // per (group, slot): how to transform raw column -> model input
  int src;           // source column or -1 (zero fill)
  float fill;        // NaN/inf replacement (train nanmean)
  float lo, hi;      // soft outlier bounds (or -inf/+inf when disabled)
  float mean, sd;    // train z-score (sd already includes the +1e-20)
  float scale;       // 1 if the slot's column is used (non-constant after normalisation), else 0
};
// encoder statistics of one member: x-encoder slots [G * fpg] (train rows [0, N) of S) and the label mean
// ymean[0] over y[0, ny), one launch
hipError_t launch_encode_stats(const float* x /*[S][F]*/, int S, int F, int N, int G, int fpg, float sigma,
                               SlotParams* slots, const float* y, int ny, float* ymean, hipStream_t st);
// the member's input state X [T][S][E] (T = G + C + 1), fp32 or fp16 (f16): x tokens from the slots, mixer
// tokens + positional rows, the label token (labels y[0, N); rows >= N are test rows); NaN -> flag bits 1 / 2
hipError_t launch_assemble(const float* x, int S, int F, int G, int fpg, int nf, const SlotParams* slots,
                           const float* w_enc /*[E][2nf]*/, const float* posemb /*[G+C][E]*/,
                           const float* tok /*[S][C][E]*/, int C, const float* y, int N, const float* uniq, int U,
                           const float* yw /*[E][2]*/, const float* yb, const float* ymean, void* X, bool f16, int E,
                           int* flag, hipStream_t st);
hipError_t launch_pos_emb(const float* rnd /*[n][E/4]*/, int n, const float* w /*[E][E/4]*/,
                          const float* b, float* out /*[n][E]*/, int E, hipStream_t st);
// M members' decoders: X + m*xm [Q][E] -> out + m*om [Q][n_out]; scratch >= M*(Fh/64)*Q*n_out floats
hipError_t launch_decoder(const float* X /*[Q][E]*/, int Q, const float* w1t /*[E][Fh]*/, const float* b1, int Fh,
                          const float* w2, const float* b2, int n_out, float* out, int E, hipStream_t st, int M,
                          int64_t xm, int64_t om, float* scratch);

// the 16-bit modes' decoder on MFMA: X fp32 (bf16 operands) or fp16 (x_f16, fp16 operands); W1 [Fh][E] and W2p
// [16][Fh] (pack_mlp2_perm order, rows >= n_out zero) in the operand type; Fh % 128 == 0, n_out <= 16
hipError_t launch_decoder_mfma(const void* X, bool x_f16, int Q, const void* W1, const float* b1, int Fh, const void* W2p,
                               const float* b2, int n_out, float* out, int E, hipStream_t st, int M, int64_t xm,
                               int64_t om);
// PREC_F16 state conversions: nb blocks of per_block elements (per_block % 4 == 0) at the given block
// strides (elements); the state [T][S][E] fp16 -> the reference order [S][T][E] fp32
hipError_t launch_f32_to_f16(const float* in, int64_t in_bstride, void* out, int64_t out_bstride, int64_t per_block,
                             int nb, hipStream_t st);
hipError_t launch_f16_to_f32(const void* in, int64_t in_bstride, float* out, int64_t out_bstride, int64_t per_block,
                             int nb, hipStream_t st);
hipError_t launch_state_f16_to_f32(const void* X, float* out, int S, int T, int E, hipStream_t st);

hipError_t launch_aggregate(const float* logits /*[M][Q][n_out]*/, int M, int Q, int n_out,
                            const int* perms /*[M][n_cls] or null*/, int n_cls, float temp, int avg_before,
                            const float* class_weights /*[n_cls] or null*/, float* probs, hipStream_t st);

// ---- mixer helpers -----------------------------------------------------------------
hipError_t launch_layernorm_rows(const float* in, int64_t rows, int dim, float eps, void* out, bool out_f32,
                                 const float* gamma, const float* beta, hipStream_t st, bool out_f16 = false);
hipError_t launch_cap_attention(const float* qp /*[cap][E]*/, const void* kv /*[S][M][2E]*/, bool kv_f32,
                                void* out /*[S][cap][E] fp32, or bf16 (out_bf16)*/, bool out_bf16, int S, int M, int cap,
                                int E, hipStream_t st);
// CAP core on MFMA (bf16; head dim 8, 24 heads = cap queries, M % 32 == 0, M <= 128): K [S*M][E], V^T [S][E][M]
// bf16 (launch_rowgemm_ln_store's transposed form), O bf16 [S][cap][E]; hipErrorNotSupported for other shapes
hipError_t launch_cap_attention_mfma(const float* qp, const void* K, const void* VT, void* out, int S, int M, int cap,
                                     int E, hipStream_t st);
// CAP tail (mlp_rows.hip, E = 192): out = LN(o2) g + b + FFN(o2), o2 = O Wout^T + bo, over M pooled tokens; O bf16,
// Wout [E][E] bf16, W1perm / W2perm the FFN in mlp_rows order (pack_mlp1_perm / pack_mlp2_perm), vecs = [bo | b0 | g |
// b + b3] fp32 (5E floats)
hipError_t launch_cap_tail(const void* O, const void* Wout, const void* W1perm, const void* W2perm, const float* vecs,
                           float* out, int64_t M, int E, float eps, hipStream_t st);
hipError_t launch_ln_add(const float* o, const float* f, const float* g, const float* b, float* out,
                         int64_t rows, int E, float eps, hipStream_t st);
hipError_t launch_gate_softmax(const float* x /*[S][D]*/, int64_t ldx, int S, int D, const float* w /*[n][D]*/,
                               const float* b, int n, float* probs, hipStream_t st);
hipError_t launch_scale_tokens(float* tok /*[S][n][E]*/, const float* probs /*[S][n]*/, int S, int n, int E,
                               hipStream_t st);

}  // namespace mmpfn
