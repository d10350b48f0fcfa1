/*
 * mmpfn_hip.h -- C ABI of the MI355X (gfx950) MMPFN in-context inference engine.
 *
 * Plain pointers and sizes only (no torch types).  All data pointers are DEVICE
 * pointers unless a parameter says "host".  The caller owns input/output buffers;
 * the context owns packed weights and workspace.  Calls on one context are
 * serialised on its stream and are asynchronous unless documented otherwise.
 *
 * Reference interfaces replaced (paths under too-z/MultiModalPFN/mmpfn/models/mmpfn/):
 *   mmpfn_create / mmpfn_set_model / mmpfn_load_weight / mmpfn_finalize_weights
 *       <- model/loading.py:401-542  load_model(): PerFeatureTransformer(...) +
 *          model.load_state_dict(state_dict, strict=False)
 *   mmpfn_mixer_forward
 *       <- model/transformer.py:755-761  self.mgm / self.cap / self.moe applied to image
 *          (MultiheadGatedMLP :33-57, CrossAttentionPooler :60-88, MoE :91-128)
 *   mmpfn_forward
 *       <- model/transformer.py:462-545,555-867  PerFeatureTransformer.forward(
 *          None, X_full[S,1,F], image_full, y_train[N], single_eval_pos=N,
 *          only_return_standard_out=True) as called at inference.py:343-348
 *   mmpfn_embed / mmpfn_run_layers / mmpfn_decode / mmpfn_copy_state
 *       <- the same forward split at its seams (embedded_input :788,
 *          transformer_encoder :799-808, decoder :850-853) for parity taps
 *   mmpfn_item_attention
 *       <- model/layer.py:341-379 attn_between_items (one token column batch)
 *   mmpfn_item_attention_layer
 *       <- model/layer.py:341-379 attn_between_items of one layer: train rows
 *          (:362-372) and test rows against head 0's K/V (:344-358) together
 *   mmpfn_item_attention_cached
 *       <- model/layer.py:344-358 with multi_head_attention.py:461-472: test rows of
 *          every head against the cached head-0 K/V of the train rows (fit_with_cache)
 *   mmpfn_status
 *       <- model/transformer.py:727-731,790-796 NaN checks (ValueError)
 *   mmpfn_feature_attention / mmpfn_item_attention_block / mmpfn_mlp_ln
 *       <- model/layer.py:332-339 / :341-379 / :410-424 with the post-norms :437-455
 *          (one PerFeatureEncoderLayer sublayer each)
 *   mmpfn_mgm / mmpfn_cap
 *       <- model/transformer.py:33-57 MultiheadGatedMLP / :60-88 CrossAttentionPooler
 */
#ifndef MMPFN_HIP_H_
#define MMPFN_HIP_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MMPFN_OK 0
#define MMPFN_ERR_INVALID (-1)   /* bad argument / shape */
#define MMPFN_ERR_HIP (-2)       /* HIP runtime error (see mmpfn_last_error) */
#define MMPFN_ERR_NAN (-3)       /* NaN in the embedded input (reference raises ValueError) */
#define MMPFN_ERR_STATE (-4)     /* call order (weights not finalised, ...) */
#define MMPFN_ERR_WEIGHT (-5)    /* missing / mis-shaped weight */

#define MMPFN_PREC_F32 0      /* parity mode: fp32 tensors; contractions on bf16 MFMA with every operand split into
                                  bf16 hi + lo planes (hi.hi + hi.lo + lo.hi, fp32 accumulate: ~2^-16 relative) */
#define MMPFN_PREC_BF16 1     /* performance mode: bf16 MFMA operands, fp32 accumulate / residual / LN */
#define MMPFN_PREC_F32_MFMA 2 /* parity mode on fp32-input MFMA (exact fp32 fma chains, 1/16 of the bf16 rate) */
#define MMPFN_PREC_BF16_F8 3  /* MMPFN_PREC_BF16 with the sample-axis attention's P.V and row sums on block-scaled fp8
                                  MFMA (V^T e4m3, P e4m3 under a per-query power-of-two scale): config E's fp8 path
                                  (multi_head_attention.py:693-729 in fp8); the train-KV cache keeps bf16 */
#define MMPFN_PREC_BF16_F8E5 4 /* as MMPFN_PREC_BF16_F8 with P in e5m2 (wider range, 2 mantissa bits) */
#define MMPFN_PREC_F16 5      /* the reference's fp16 autocast (utils.py:150-190, layer.py:60-62): the state X kept in
                                  fp16 between kernels, every layer contraction on fp16 MFMA operands (the item
                                  attention's Q / K and P.V on bf16), fp32 accumulation / LayerNorm / softmax
                                  statistics; tables of more than 64 tokens per row run MMPFN_PREC_BF16 */
#define MMPFN_PREC_F16_F8 6   /* MMPFN_PREC_F16 with the fp8 P.V of MMPFN_PREC_BF16_F8 */
#define MMPFN_PREC_F16_F8E5 7 /* MMPFN_PREC_F16 with the fp8 P.V of MMPFN_PREC_BF16_F8E5 */

#define MMPFN_MIXER_NONE 0
#define MMPFN_MIXER_MGM 1
#define MMPFN_MIXER_MGM_CAP 2
#define MMPFN_MIXER_MOE 3

typedef struct mmpfn_ctx mmpfn_ctx;

typedef struct mmpfn_model_desc {
  int emsize;             /* E = 192 */
  int nhead;              /* 6 (head dim must be 32) */
  int nlayers;            /* 12 */
  int nhid;               /* 768 (MLP hidden, decoder hidden, modality width) */
  int features_per_group; /* model grouping (yaml) */
  int encoder_features;   /* encoder width nf (checkpoint config.features_per_group) */
  int n_out;              /* decoder outputs (10) */
  int mixer_type;         /* MMPFN_MIXER_* */
  int mgm_heads;          /* MGM heads, or MoE experts */
  int cap_heads;          /* CAP queries/heads */
  int two_sets_of_queries;
  int remove_duplicate_features; /* encoder Linear step index 6 instead of 5 */
  float ln_eps;           /* 1e-5 */
  float outlier_sigma;    /* 12 for classification; <= 0 disables soft clipping */
} mmpfn_model_desc;

/* ---- lifecycle ------------------------------------------------------------------ */
mmpfn_ctx* mmpfn_create(int device, void* hip_stream);
void mmpfn_destroy(mmpfn_ctx* ctx);
const char* mmpfn_last_error(const mmpfn_ctx* ctx);
int mmpfn_set_stream(mmpfn_ctx* ctx, void* hip_stream);
const char* mmpfn_version(void);

/* ---- weights (checkpoint ABI: reference state_dict names, fp32 host data) -------- */
int mmpfn_set_model(mmpfn_ctx* ctx, const mmpfn_model_desc* desc);
int mmpfn_load_weight(mmpfn_ctx* ctx, const char* name, const float* host_data, int64_t numel);
int mmpfn_finalize_weights(mmpfn_ctx* ctx); /* pack / fold / convert / upload; synchronous */

/* ---- modality projection heads --------------------------------------------------
 * image [S][n_mod][nhid] -> tokens [S][C][E]; C = mmpfn_mixer_tokens(ctx, n_mod). */
int mmpfn_mixer_tokens(const mmpfn_ctx* ctx, int n_mod);
int mmpfn_mixer_forward(mmpfn_ctx* ctx, const float* image, int S, int n_mod, float* tokens, int precision);

/* ---- one ensemble member's forward ------------------------------------------------
 * x        [S][F] fp32 (NULL when tabular input is absent)
 * tokens   [S][C][E] mixer tokens (NULL / C = 0 when there is no image)
 * y_train  [N] fp32 class codes; uniq [U] sorted unique train codes (after NaN fill)
 * pos_rand [G + C][E/4]: torch.randn from the model's CPU generator
 *          (transformer.py:421-424,925-931), G = ceil(F / features_per_group)
 * logits   [S - N][n_out] fp32 output                                               */
int mmpfn_forward(mmpfn_ctx* ctx, const float* x, int S, int F, const float* tokens, int C, const float* y_train,
                  int N, const float* uniq, int U, const float* pos_rand, float* logits, int precision);

/* forward split at its seams (parity taps) */
int mmpfn_embed(mmpfn_ctx* ctx, const float* x, int S, int F, const float* tokens, int C, const float* y_train, int N,
                const float* uniq, int U, const float* pos_rand, int precision);
int mmpfn_run_layers(mmpfn_ctx* ctx, int layer_begin, int layer_end);
int mmpfn_decode(mmpfn_ctx* ctx, float* logits);
/* copies the current state in reference order [S][T][E] (fp32) */
int mmpfn_copy_state(mmpfn_ctx* ctx, float* out, int64_t capacity_elems);
int mmpfn_state_tokens(const mmpfn_ctx* ctx); /* T of the current state */

/* Ensemble aggregation (classifier.py:541-566, replaces the torch post-processing):
 * logits [M][Q][n_out]; perms [M][n_cls] int32 (NULL: no class permutation);
 * temperature != 1 slices to n_cls and divides; average_before_softmax 0/1;
 * class_weights [n_cls] (balance_probabilities) or NULL; probs [Q][C] with
 * C = n_cls when sliced or permuted, else n_out. */
int mmpfn_aggregate(mmpfn_ctx* ctx, const float* logits, int M, int Q, int n_out, const int* perms, int n_cls,
                    float temperature, int average_before_softmax, const float* class_weights, float* probs);

/* Synchronises the context stream and reports deferred device-side errors
 * (MMPFN_ERR_NAN when the embedded input held NaNs). */
int mmpfn_status(mmpfn_ctx* ctx);

/* ---- raw kernels (benchmarks / unit parity) ------------------------------------
 * Sample-axis attention for one layout batch:
 *   q  [T][H][S][32], k [T][H][Npad][32], vt [T][H][32][Npad], out [T][S][H*32]
 *   queries s in [s0, s0+nq) attend keys [0, nk); kv_head_fixed >= 0 forces a KV head.
 *   softmax(q k^T / sqrt(32)): q as projected (the engine's own bf16 forward passes q pre-multiplied
 *   by log2(e)/sqrt(32) internally; these taps do not).
 * Element type: fp32 (MMPFN_PREC_F32) or bf16 (MMPFN_PREC_BF16). */
int mmpfn_item_attention(mmpfn_ctx* ctx, const void* q, const void* k, const void* vt, void* out, int S, int T,
                         int H, int Npad, int s0, int nq, int nk, int kv_head_fixed, int precision);

/* M ensemble members of one geometry (same S, N, F, C) in one batched forward: the
 * state of all members is stacked [M][T][S][E] so every layer kernel runs once over the
 * batch (M*S rows, M*T attention columns).  x, y, uniq: HOST arrays of M device pointers
 * (as mmpfn_forward's arguments of each member); U: host array of M unique-label counts;
 * logits: device [M][S-N][n_out].  Replaces the per-member model call of the ensemble loop
 * (inference.py:294-349 -> transformer.py:462-545) for members that share a geometry. */
int mmpfn_forward_batch(mmpfn_ctx* ctx, int M, const float* const* x, int S, int F, const float* tokens, int C,
                        const float* const* y, int N, const float* const* uniq, const int* U,
                        const float* pos_rand, float* logits, int precision);

/* Forward lanes: independent per-member workspaces sharing the context's weights.
 * Selects the lane used by the following embed / run_layers / decode / forward /
 * copy_state calls (lane 0 at creation).  Members run concurrently when the caller binds a
 * different stream (mmpfn_set_stream) to each lane; mmpfn_status checks every lane.
 * Replaces nothing in the reference: its ensemble loop runs members one after another
 * (inference.py:294-349); lanes let independent members overlap on one GPU. */
#define MMPFN_MAX_LANES 8
int mmpfn_select_lane(mmpfn_ctx* ctx, int lane);

/* The whole sample-axis attention of one layer in one launch (bf16 only): train queries
 * s in [0, N) of head h against K/V head h, test queries s in [N, S) of every head against
 * K/V head 0; keys [0, N).  Layouts as mmpfn_item_attention. */
int mmpfn_item_attention_layer(mmpfn_ctx* ctx, const void* q, const void* k, const void* vt, void* out, int S,
                               int T, int H, int Npad, int N);

/* mmpfn_item_attention_layer in a 16-bit precision code: MMPFN_PREC_BF16 (as mmpfn_item_attention_layer),
 * MMPFN_PREC_F16 (q, k and out in fp16, vt bf16), or either with the fp8 P.V (MMPFN_PREC_*_F8: P e4m3,
 * *_F8E5: P e5m2; vt is the bf16 V^T, converted to e4m3 inside).  A code 5-7 OR MMPFN_ATTN_QK_BF16 runs the
 * fp16 mode's forward form: q and k in bf16 (as the engine writes them), out fp16. */
#define MMPFN_ATTN_QK_BF16 0x100
int mmpfn_item_attention_layer_ex(mmpfn_ctx* ctx, const void* q, const void* k, const void* vt, void* out, int S,
                                  int T, int H, int Npad, int N, int precision);

/* The train-KV cache's attention (bf16 only): queries s in [0, S) of every head against a
 * head-0-only K [T][Npad][32] / V^T [T][32][Npad] (the layout mmpfn_cache_build keeps per
 * layer); keys [0, N).  Q / out as mmpfn_item_attention. */
int mmpfn_item_attention_cached(mmpfn_ctx* ctx, const void* q, const void* k0, const void* vt0, void* out, int S,
                                int T, int H, int Npad, int N);

/* Train-KV cache (fit_mode="fit_with_cache"), one per ensemble member.
 * mmpfn_cache_build: forward of the N train rows only (x [N][F], tokens [N][C][E], y_train [N]);
 *   keeps, per layer, head 0's K and V^T of the train rows -- the only K/V the test rows read
 *   (multiquery item attention, layer.py:341-358; only_cache_first_head_kv, :362-372) -- and the
 *   train statistics of the x / y encoders and the positional embeddings.  Replaces
 *   InferenceEngineCacheKV.prepare's ens_model.forward(..., single_eval_pos=len(X))
 *   (inference.py:425-436; cache_kv=True, multi_head_attention.py:461-472).
 * mmpfn_cache_predict: Q test rows (x [Q][F], tokens [Q][C][E]) through the layers against the
 *   cache (use_cached_kv, layer.py:344-358), logits [Q][n_out] in the cache's precision.  Replaces
 *   iter_outputs' model(None, X_test, None, single_eval_pos=None) (inference.py:499-507).
 * Equal to the test rows of a full forward over train + test rows, except that the x encoder's
 * constant-column and used-feature tests see the train rows only (as the reference's cache).
 * The cache belongs to the context that built it; free it with mmpfn_cache_free. */
typedef struct mmpfn_cache mmpfn_cache;
int mmpfn_cache_build(mmpfn_ctx* ctx, const float* x, int N, int F, const float* tokens, int C, const float* y_train,
                      const float* uniq, int U, const float* pos_rand, int precision, mmpfn_cache** out);
int mmpfn_cache_predict(mmpfn_ctx* ctx, const mmpfn_cache* cache, const float* x, int Q, int F, const float* tokens,
                        int C, float* logits);
int64_t mmpfn_cache_bytes(const mmpfn_cache* cache);
void mmpfn_cache_free(mmpfn_ctx* ctx, mmpfn_cache* cache);

/* Measurement hook (no reference counterpart): while enabled, every sample-axis attention
 * launch of the bf16 forward is bracketed by HIP events on its own stream.  enable=1 clears
 * and starts a window, enable=0 stops it; _read synchronises and returns the summed launch
 * durations, the launch count and their algorithmic flops (4*T*(N+Q)*N*E each). */
int mmpfn_kernel_timing(mmpfn_ctx* ctx, int enable);
int mmpfn_kernel_timing_read(mmpfn_ctx* ctx, double* total_ms, int64_t* launches, double* flops);

/* Parity mode (PREC_F32): the item attention's key count from which it runs the measured precision budget's
 * cheap forms instead of three split products -- an opt-in throughput mode (about 1.2x the parity
 * step), off by default: the sweep of logits error against N on the golden models (profiles/r06/parity_n0_sweep_
 * form*.txt) found no N from which the cheap forms keep the 1e-4 contract (multi_head_attention.py:718-729 in fp32)
 * with 2x margin.  Process-wide; returns the previous value.  n < 0: never.  form: 1 fp16 S only, 2 two-product P.V
 * only, 3 both, 0 keep. */
int mmpfn_set_parity_attention_min_keys(int n, int form);

/* Per-sublayer taps: one sublayer of layer `layer` on a caller-provided state, in place, on the
 * context stream (the forward itself fuses across these seams: the bf16 item-attention
 * out-projection runs inside the MLP kernel there).  X: device [T][S][E] fp32, the engine's
 * token-major state of ONE member (reference order [S][T][E] transposed).  `rows` = S * T. */
int mmpfn_feature_attention(mmpfn_ctx* ctx, int layer, float* X, int S, int T, int precision);
/* train rows [0, N) attend their own heads, rows [N, S) head 0's K/V (MQA) */
int mmpfn_item_attention_block(mmpfn_ctx* ctx, int layer, float* X, int S, int T, int N, int precision);
int mmpfn_mlp_ln(mmpfn_ctx* ctx, int layer, float* X, int64_t rows, int precision);
/* modality heads: image [S][n_mod][nhid] -> MGM tokens [S][mgm*n_mod][E] (head-major, as the
 * reference concatenates them); MGM tokens [S][M][E] -> CAP tokens [S][cap][E] */
int mmpfn_mgm(mmpfn_ctx* ctx, const float* image, int S, int n_mod, float* tokens, int precision);
int mmpfn_cap(mmpfn_ctx* ctx, const float* mgm_tokens, int S, int M, float* tokens, int precision);

/* Host helper of the predict path (no GPU, no context): the fingerprint feature's row hash
 * (model/preprocessing.py:476-479, Python hash(row.tobytes()) under PYTHONHASHSEED=0 = SipHash-2-4 with the
 * all-zero key, -1 mapped to -2).  rows: host, n_rows x row_bytes contiguous; out: host int64[n_rows]. */
int mmpfn_siphash24_rows(const void* rows, int64_t n_rows, int64_t row_bytes, int64_t* out);

#ifdef __cplusplus
}
#endif

#endif /* MMPFN_HIP_H_ */
