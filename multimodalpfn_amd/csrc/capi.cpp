// C ABI of the MMPFN engine: context, weight packing (checkpoint ABI) and the
// native orchestration of one ensemble member's PerFeatureTransformer forward.
//
// Forward (transformer.py:555-867) per member, all on the context stream:
//   pos-emb  -> x encoder (+pos-emb) -> mixer tokens (+pos-emb) -> y token
//   -> nlayers x [feature attn | item attn | MLP] (layer.py:272-457)
//   -> decoder on the test rows of the target token.
// State layout in HBM: X[T][S][E] fp32 (token-major), so every token column of the
// sample-axis attention is a contiguous [S][E] slab; fp16 under PREC_F16 (the encoders and the
// decoder run in fp32 and convert at the seams).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <utility>
#include <vector>

#include "../../include/mmpfn_hip.h"
#include "kernels.h"
#include "weight_pack.h"

using namespace mmpfn;

namespace {

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  size_t n = 0;  // elements (split weight planes: elements per plane)
};

struct LayerW {  // packed per layer, [N][K] row-major
  DevBuf feat_qkv, feat_out, item_qkv, item_qtest, item_out, mlp1, mlp2;  // fp32
  DevBuf feat_qkv_h, feat_out_h, item_qkv_h, item_qtest_h, item_out_h, mlp1_h, mlp2_h;  // bf16
  DevBuf feat_pack_h;  // bf16 LDS images of the feature-attention weights (featrow.hip)
  // PREC_F16 (fp16): feature-attention images (out-projection rows in f16_row_perm order), item q|k|v and
  // test q (Q rows prescaled like the bf16 copies), item out-projection and MLP W2 with f16_row_perm rows,
  // MLP W1 natural
  DevBuf feat_pack_f, item_qkv_f, item_qtest_f, item_out_f, mlp1_f, mlp2_f;
};

}  // namespace

// train-KV cache of one ensemble member (fit_mode="fit_with_cache"): per layer the head-0 K and
// V^T of the train rows (all test rows read, layer.py:344-358), plus the train statistics of the
// input encoders and the positional embeddings, so a predict runs only the test rows
struct mmpfn_cache {
  int N = 0, F = 0, G = 0, C = 0, T = 0, Npad = 0, prec = 0, U = 0;
  DevBuf kv;     // [L][K: T x Npad x 32 | V^T: T x 32 x Npad], element size of prec
  DevBuf slots;  // x-encoder SlotParams [G * fpg]
  DevBuf ymean;  // y-encoder train nanmean
  DevBuf uniq;   // sorted unique train labels [U]
  DevBuf pe;     // positional embeddings [G + C][E]
};

struct mmpfn_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  // every stream bound since the last mmpfn_status: lanes run on their own streams and the NaN
  // flags they set must be read behind all of them
  std::vector<hipStream_t> seen_streams;
  std::string err;
  bool have_model = false, finalized = false;
  mmpfn_model_desc d{};
  std::map<std::string, std::vector<float>> host;
  std::vector<DevBuf> owned;

  std::vector<LayerW> layers;
  // parity mode (PREC_F32): every GEMM weight also as bf16 hi | lo planes, keyed by its fp32 copy
  std::map<const void*, DevBuf> split;
  DevBuf enc_w, y_w, y_b, pe_w, pe_b, dec_w1, dec_b1, dec_w2, dec_b2;
  DevBuf dec_w1_h, dec_w1_f, dec_w2p_h, dec_w2p_f;  // 16-bit decoder: W1 [Fh][E], W2 [16][Fh] permuted
  // mixer
  DevBuf mgm_w1, mgm_w1_h, mgm_w1_f, mgm_b1, mgm_w2, mgm_w2_h, mgm_w2_f, mgm_b2;
  DevBuf cap_qp, cap_kv, cap_kv_h, cap_kv_b, cap_o, cap_o_h, cap_o_b, cap_f0, cap_f0_h, cap_f0_b, cap_f3, cap_f3_h,
      cap_f3_b, cap_ng, cap_nb;
  DevBuf cap_f0_p, cap_f3_p, cap_vecs;  // E = 192: the FFN in mlp_rows order (bf16) and [bo | b0 | g | b + b3]
  DevBuf moe_w1, moe_w1_h, moe_b1, moe_w2, moe_w2_h, moe_b2, moe_gw, moe_gb;

  // workspace of the selected lane (per-member forward state)
  DevBuf ws_X, ws_O, ws_big, ws_pe, ws_slots, ws_scr, ws_flag;
  DevBuf mx[8];
  DevBuf tap_v8;   // e4m3 V^T of the fp8 attention tap
  DevBuf tap_x16;  // PREC_F16 taps: the caller's fp32 state as fp16
  // current forward geometry (M members of equal geometry stacked as [M][T][S][E]); f8: the fp8 P.V
  // variant of the item attention (f8_of of the forward's precision code; prec holds its base_prec)
  int S = 0, T = 0, N = 0, G = 0, C = 0, Npad = 0, prec = 0, M = 1, f8 = 0;
  bool embedded = false;
  // lanes: independent forward workspaces sharing the weights, so members can run
  // concurrently on different streams; the selected lane lives in the fields above and the
  // others are parked here (mmpfn_select_lane swaps them)
  struct Lane {
    DevBuf ws_X, ws_O, ws_big, ws_pe, ws_slots, ws_scr, ws_flag;
    int S = 0, T = 0, N = 0, G = 0, C = 0, Npad = 0, prec = 0, M = 1, f8 = 0;
    bool embedded = false;
  };
  std::vector<Lane> lanes;  // lanes[cur] is stale while cur is selected
  int cur = 0;
  // live timing of the sample-axis attention launches (mmpfn_kernel_timing): HIP events
  // recorded on the launching stream around every item-attention launch while enabled
  mmpfn_cache* cache_out = nullptr;       // being built by the current forward (train rows only)
  const mmpfn_cache* cache_in = nullptr;  // used by the current forward (test rows only)
  bool kt_on = false;
  std::vector<hipEvent_t> kt_pool;  // event pairs, reused across windows
  size_t kt_used = 0;
  double kt_flops = 0.0;
  template <typename A, typename B>
  static void swap_lane(A& a, B& b) {
    std::swap(a.ws_X, b.ws_X), std::swap(a.ws_O, b.ws_O), std::swap(a.ws_big, b.ws_big);
    std::swap(a.ws_pe, b.ws_pe), std::swap(a.ws_slots, b.ws_slots), std::swap(a.ws_scr, b.ws_scr);
    std::swap(a.ws_flag, b.ws_flag);
    std::swap(a.S, b.S), std::swap(a.T, b.T), std::swap(a.N, b.N), std::swap(a.G, b.G), std::swap(a.C, b.C);
    std::swap(a.Npad, b.Npad), std::swap(a.prec, b.prec), std::swap(a.embedded, b.embedded), std::swap(a.M, b.M);
    std::swap(a.f8, b.f8);
  }
};

namespace {

int fail(mmpfn_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}

#define HIPCHK(expr)                                                                          \
  do {                                                                                        \
    hipError_t e_ = (expr);                                                                   \
    if (e_ != hipSuccess) return fail(ctx, MMPFN_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

#define RC_(expr)                    \
  do {                               \
    int rc_ = (expr);                \
    if (rc_ != MMPFN_OK) return rc_; \
  } while (0)

// the shapes the fp16 MGM head bank's big-tile kernels take (uploaded by finalize, used by mixer_mgm)
bool mgm_f16_shape(const mmpfn_model_desc& d) {
  return d.emsize == 192 && (d.mgm_heads * d.nhid) % 256 == 0 && d.nhid % 64 == 0;
}

int ensure(mmpfn_ctx* ctx, DevBuf& b, size_t bytes) {
  if (b.bytes >= bytes && b.p) return MMPFN_OK;
  if (b.p) HIPCHK(hipFree(b.p));
  b.p = nullptr;
  b.bytes = 0;
  bytes = (bytes + 255) & ~size_t(255);
  HIPCHK(hipMalloc(&b.p, bytes));
  b.bytes = bytes;
  return MMPFN_OK;
}

// the lane's NaN flag: zeroed once when allocated, then only ORed into by the encoder kernels and
// cleared by mmpfn_status after it has been read, so a NaN in ANY forward queued on the lane since
// the last status check is reported (not only the last forward's)
int ensure_flag(mmpfn_ctx* ctx, DevBuf& b, hipStream_t st) {
  if (b.p) return MMPFN_OK;
  RC_(ensure(ctx, b, 256));
  HIPCHK(hipMemsetAsync(b.p, 0, 256, st));
  return MMPFN_OK;
}

// fp16 copy (PREC_F16 weights)
int upload_f16(mmpfn_ctx* ctx, DevBuf& b, const std::vector<float>& v) {
  std::vector<uint16_t> h(v.size());
  for (size_t i = 0; i < v.size(); ++i) h[i] = f2h(v[i]);
  int rc = ensure(ctx, b, h.size() * 2);
  if (rc) return rc;
  HIPCHK(hipMemcpy(b.p, h.data(), h.size() * 2, hipMemcpyHostToDevice));
  return MMPFN_OK;
}

int upload(mmpfn_ctx* ctx, DevBuf& b, const std::vector<float>& v, bool as_bf16) {
  if (as_bf16) {
    std::vector<uint16_t> h(v.size());
    for (size_t i = 0; i < v.size(); ++i) h[i] = f2bf(v[i]);
    int rc = ensure(ctx, b, h.size() * 2);
    if (rc) return rc;
    HIPCHK(hipMemcpy(b.p, h.data(), h.size() * 2, hipMemcpyHostToDevice));
  } else {
    int rc = ensure(ctx, b, v.size() * 4);
    if (rc) return rc;
    HIPCHK(hipMemcpy(b.p, v.data(), v.size() * 4, hipMemcpyHostToDevice));
  }
  return MMPFN_OK;
}

const std::vector<float>* getw(mmpfn_ctx* ctx, const std::string& name, size_t numel) {
  auto it = ctx->host.find(name);
  if (it == ctx->host.end()) {
    ctx->err = "missing weight: " + name;
    return nullptr;
  }
  if (it->second.size() != numel) {
    ctx->err = "weight " + name + " has " + std::to_string(it->second.size()) + " elements, expected " +
               std::to_string(numel);
    return nullptr;
  }
  return &it->second;
}

#define GETW(var, name, n)                                  \
  const std::vector<float>* var = getw(ctx, (name), (n));  \
  if (!var) return MMPFN_ERR_WEIGHT;

// bf16 hi | lo planes of v (hi = bf16(w), lo = bf16(w - hi)), the weight operand of the parity mode's
// three-product GEMMs, stored under the key of its fp32 copy f
int upsplit(mmpfn_ctx* ctx, const DevBuf& f, const std::vector<float>& v) {
  std::vector<uint16_t> h(2 * v.size());
  for (size_t i = 0; i < v.size(); ++i) {
    const uint16_t hi = f2bf(v[i]);
    uint32_t u = (uint32_t)hi << 16;
    float fh;
    std::memcpy(&fh, &u, 4);
    h[i] = hi;
    h[v.size() + i] = f2bf(v[i] - fh);
  }
  DevBuf& b = ctx->split[f.p];
  int rc = ensure(ctx, b, h.size() * 2);
  if (rc) return rc;
  b.n = v.size();
  HIPCHK(hipMemcpy(b.p, h.data(), h.size() * 2, hipMemcpyHostToDevice));
  return MMPFN_OK;
}

int up2(mmpfn_ctx* ctx, DevBuf& f, DevBuf& h, const std::vector<float>& v) {
  int rc = upload(ctx, f, v, false);
  if (rc) return rc;
  if ((rc = upload(ctx, h, v, true))) return rc;
  return upsplit(ctx, f, v);
}

int finalize(mmpfn_ctx* ctx) {
  const mmpfn_model_desc& d = ctx->d;
  const int E = d.emsize, HD = E, Fh = d.nhid, nf = d.encoder_features;
  ctx->layers.assign(d.nlayers, LayerW{});
  for (int l = 0; l < d.nlayers; ++l) {
    const std::string p = "transformer_encoder.layers." + std::to_string(l) + ".";
    LayerW& L = ctx->layers[l];
    int rc;
    GETW(fq, p + "self_attn_between_features._w_qkv", (size_t)3 * HD * E);
    GETW(fo, p + "self_attn_between_features._w_out", (size_t)HD * E);
    GETW(io, p + "self_attn_between_items._w_out", (size_t)HD * E);
    GETW(m1, p + "mlp.linear1.weight", (size_t)Fh * E);
    GETW(m2, p + "mlp.linear2.weight", (size_t)E * Fh);
    if ((rc = up2(ctx, L.feat_qkv, L.feat_qkv_h, *fq))) return rc;
    if ((rc = up2(ctx, L.feat_out, L.feat_out_h, transpose_out(*fo, HD, E)))) return rc;
    if (E == 192 && d.nhead == 6) {
      if ((rc = upload(ctx, L.feat_pack_h, pack_feat_rows(*fq, transpose_out(*fo, HD, E), d.nhead, E), true)))
        return rc;
      if ((rc = upload_f16(ctx, L.feat_pack_f, pack_feat_rows(*fq, transpose_out(*fo, HD, E), d.nhead, E, true))))
        return rc;
      if ((rc = upload_f16(ctx, L.item_out_f, permute_rows_f16(transpose_out(*io, HD, E), E, HD)))) return rc;
      if ((rc = upload_f16(ctx, L.mlp1_f, *m1))) return rc;
      if ((rc = upload_f16(ctx, L.mlp2_f, permute_rows_f16(pack_mlp2_perm(*m2, E, Fh), E, Fh)))) return rc;
    }
    if ((rc = up2(ctx, L.item_out, L.item_out_h, transpose_out(*io, HD, E)))) return rc;
    if ((rc = upload(ctx, L.mlp1, *m1, false))) return rc;
    if ((rc = upsplit(ctx, L.mlp1, *m1))) return rc;
    if ((rc = upload(ctx, L.mlp1_h, E == 192 ? pack_mlp1_perm(*m1, E, Fh) : *m1, true))) return rc;
    if ((rc = upload(ctx, L.mlp2, *m2, false))) return rc;
    if ((rc = upsplit(ctx, L.mlp2, *m2))) return rc;
    if ((rc = upload(ctx, L.mlp2_h, pack_mlp2_perm(*m2, E, Fh), true))) return rc;
    if ((rc = upsplit(ctx, L.mlp2_h, pack_mlp2_perm(*m2, E, Fh)))) return rc;  // parity mode (mlp_x3_kernel)
    std::vector<float> wtrain((size_t)3 * HD * E), wtest((size_t)HD * E);
    if (d.two_sets_of_queries) {
      GETW(wq, p + "self_attn_between_items._w_q", (size_t)2 * HD * E);
      GETW(wkv, p + "self_attn_between_items._w_kv", (size_t)2 * HD * E);
      std::copy(wq->begin(), wq->begin() + (size_t)HD * E, wtrain.begin());
      std::copy(wkv->begin(), wkv->end(), wtrain.begin() + (size_t)HD * E);
      std::copy(wq->begin() + (size_t)HD * E, wq->end(), wtest.begin());
    } else {
      GETW(wqkv, p + "self_attn_between_items._w_qkv", (size_t)3 * HD * E);
      wtrain = *wqkv;
      std::copy(wqkv->begin(), wqkv->begin() + (size_t)HD * E, wtest.begin());
    }
    if ((rc = upload(ctx, L.item_qkv, wtrain, false))) return rc;
    if ((rc = upload(ctx, L.item_qtest, wtest, false))) return rc;
    if ((rc = upsplit(ctx, L.item_qkv, wtrain))) return rc;
    if ((rc = upsplit(ctx, L.item_qtest, wtest))) return rc;
    // bf16 copies: the Q rows carry the attention kernel's log2(e)/sqrt(32) (attn_pipe_kernel with
    // q_prescaled: no per-query scaling pass; one bf16 rounding of Q instead of two)
    const float qsc = 1.4426950408889634f / std::sqrt((float)(E / d.nhead));
    for (size_t i = 0; i < (size_t)HD * E; ++i) wtrain[i] *= qsc;
    for (float& w : wtest) w *= qsc;
    if ((rc = upload(ctx, L.item_qkv_h, wtrain, true))) return rc;
    if ((rc = upload(ctx, L.item_qtest_h, wtest, true))) return rc;
    if ((rc = upload_f16(ctx, L.item_qkv_f, wtrain))) return rc;
    if ((rc = upload_f16(ctx, L.item_qtest_f, wtest))) return rc;
  }
  int rc;
  {
    const std::string en = d.remove_duplicate_features ? "encoder.6.layer.weight" : "encoder.5.layer.weight";
    GETW(w, en, (size_t)E * 2 * nf);
    if ((rc = upload(ctx, ctx->enc_w, *w, false))) return rc;
    GETW(yw, "y_encoder.2.layer.weight", (size_t)E * 2);
    GETW(yb, "y_encoder.2.layer.bias", (size_t)E);
    if ((rc = upload(ctx, ctx->y_w, *yw, false))) return rc;
    if ((rc = upload(ctx, ctx->y_b, *yb, false))) return rc;
    GETW(pw, "feature_positional_embedding_embeddings.weight", (size_t)E * (E / 4));
    GETW(pb, "feature_positional_embedding_embeddings.bias", (size_t)E);
    if ((rc = upload(ctx, ctx->pe_w, *pw, false))) return rc;
    if ((rc = upload(ctx, ctx->pe_b, *pb, false))) return rc;
    GETW(dw1, "decoder_dict.standard.0.weight", (size_t)Fh * E);
    GETW(db1, "decoder_dict.standard.0.bias", (size_t)Fh);
    GETW(dw2, "decoder_dict.standard.2.weight", (size_t)d.n_out * Fh);
    GETW(db2, "decoder_dict.standard.2.bias", (size_t)d.n_out);
    if ((rc = upload(ctx, ctx->dec_w1, transpose_out(*dw1, Fh, E), false))) return rc;  // [E][Fh]
    if ((rc = upload(ctx, ctx->dec_b1, *db1, false))) return rc;
    if ((rc = upload(ctx, ctx->dec_w2, *dw2, false))) return rc;
    if ((rc = upload(ctx, ctx->dec_b2, *db2, false))) return rc;
    if (d.n_out <= 16 && Fh % 128 == 0 && E % 32 == 0 && E <= 256) {
      std::vector<float> w2p((size_t)16 * Fh, 0.f);
      std::copy(dw2->begin(), dw2->end(), w2p.begin());
      w2p = pack_mlp2_perm(w2p, 16, Fh);
      if ((rc = upload(ctx, ctx->dec_w1_h, *dw1, true))) return rc;
      if ((rc = upload_f16(ctx, ctx->dec_w1_f, *dw1))) return rc;
      if ((rc = upload(ctx, ctx->dec_w2p_h, w2p, true))) return rc;
      if ((rc = upload_f16(ctx, ctx->dec_w2p_f, w2p))) return rc;
    }
  }
  const int D = d.nhid;
  if (d.mixer_type == MMPFN_MIXER_MGM || d.mixer_type == MMPFN_MIXER_MGM_CAP) {
    const int mg = d.mgm_heads;
    std::vector<float> W1((size_t)mg * D * D), B1((size_t)mg * D), W2((size_t)mg * E * (D / 2)),
        B2((size_t)mg * E);
    for (int h = 0; h < mg; ++h) {
      const std::string p = "mgm.projs." + std::to_string(h) + ".";
      GETW(g, p + "0.weight", (size_t)D);
      GETW(b, p + "0.bias", (size_t)D);
      GETW(w1, p + "1.weight", (size_t)D * D);
      GETW(b1, p + "1.bias", (size_t)D);
      GETW(w2, p + "4.weight", (size_t)E * (D / 2));
      GETW(b2, p + "4.bias", (size_t)E);
      std::vector<float> w = *w1, c = *b1;
      fold_ln(w, c, g->data(), b->data(), D, D);
      // interleave GLU halves in 16-row blocks: [a 16i..16i+15 | b 16i..16i+15] per 32 rows
      for (int i = 0; i < D / 32; ++i)
        for (int r = 0; r < 32; ++r) {
          const int src = r < 16 ? 16 * i + r : D / 2 + 16 * i + (r - 16);
          const size_t dst = (size_t)h * D + 32 * i + r;
          std::memcpy(&W1[dst * D], &w[(size_t)src * D], D * sizeof(float));
          B1[dst] = c[src];
        }
      std::copy(w2->begin(), w2->end(), W2.begin() + (size_t)h * E * (D / 2));
      std::copy(b2->begin(), b2->end(), B2.begin() + (size_t)h * E);
    }
    if ((rc = up2(ctx, ctx->mgm_w1, ctx->mgm_w1_h, W1))) return rc;
    if ((rc = upload(ctx, ctx->mgm_b1, B1, false))) return rc;
    if ((rc = up2(ctx, ctx->mgm_w2, ctx->mgm_w2_h, W2))) return rc;
    if (mgm_f16_shape(d)) {  // PREC_F16's head bank (the big-tile kernels only)
      if ((rc = upload_f16(ctx, ctx->mgm_w1_f, W1))) return rc;
      if ((rc = upload_f16(ctx, ctx->mgm_w2_f, W2))) return rc;
    } else {  // a re-finalised context with another head count must not keep the previous model's fp16 bank
      for (DevBuf* b : {&ctx->mgm_w1_f, &ctx->mgm_w2_f})
        if (b->p) {
          HIPCHK(hipFree(b->p));
          *b = DevBuf{};
        }
    }
    if ((rc = upload(ctx, ctx->mgm_b2, B2, false))) return rc;
  }
  if (d.mixer_type == MMPFN_MIXER_MGM_CAP) {
    const int cap = d.cap_heads;
    GETW(qs, "cap.queries", (size_t)cap * E);
    GETW(qpw, "cap.q_proj.weight", (size_t)E * E);
    GETW(inw, "cap.mha.in_proj_weight", (size_t)3 * E * E);
    GETW(inb, "cap.mha.in_proj_bias", (size_t)3 * E);
    GETW(ow, "cap.mha.out_proj.weight", (size_t)E * E);
    GETW(ob, "cap.mha.out_proj.bias", (size_t)E);
    GETW(kg, "cap.k_norm.weight", (size_t)E);
    GETW(kb, "cap.k_norm.bias", (size_t)E);
    GETW(qg, "cap.q_norm.weight", (size_t)E);
    GETW(qb, "cap.q_norm.bias", (size_t)E);
    GETW(ng, "cap.out_norm.weight", (size_t)E);
    GETW(nb, "cap.out_norm.bias", (size_t)E);
    GETW(f0w, "cap.ffn.0.weight", (size_t)2 * E * E);
    GETW(f0b, "cap.ffn.0.bias", (size_t)2 * E);
    GETW(f3w, "cap.ffn.3.weight", (size_t)2 * E * E);
    GETW(f3b, "cap.ffn.3.bias", (size_t)E);
    // weight-only query path: in_proj_q(q_proj(q_norm(queries)))  (transformer.py:81)
    std::vector<float> qp((size_t)cap * E);
    for (int c = 0; c < cap; ++c) {
      const float* q = qs->data() + (size_t)c * E;
      double mu = 0, var = 0;
      for (int e = 0; e < E; ++e) mu += q[e];
      mu /= E;
      for (int e = 0; e < E; ++e) var += (q[e] - mu) * (q[e] - mu);
      var /= E;
      const double inv = 1.0 / std::sqrt(var + d.ln_eps);
      std::vector<double> qn(E), qq(E);
      for (int e = 0; e < E; ++e) qn[e] = (q[e] - mu) * inv * (*qg)[e] + (*qb)[e];
      for (int o = 0; o < E; ++o) {
        double a = 0;
        for (int e = 0; e < E; ++e) a += (*qpw)[(size_t)o * E + e] * qn[e];
        qq[o] = a;
      }
      for (int o = 0; o < E; ++o) {
        double a = (*inb)[o];
        for (int e = 0; e < E; ++e) a += (*inw)[(size_t)o * E + e] * qq[e];
        qp[(size_t)c * E + o] = (float)a;
      }
    }
    if ((rc = upload(ctx, ctx->cap_qp, qp, false))) return rc;
    // K/V in-projection with k_norm's affine folded in (k = v = k_norm(src))
    std::vector<float> wkv(inw->begin() + (size_t)E * E, inw->end());
    std::vector<float> bkv(inb->begin() + E, inb->end());
    fold_ln(wkv, bkv, kg->data(), kb->data(), 2 * E, E);
    if ((rc = up2(ctx, ctx->cap_kv, ctx->cap_kv_h, wkv))) return rc;
    if ((rc = upload(ctx, ctx->cap_kv_b, bkv, false))) return rc;
    if ((rc = up2(ctx, ctx->cap_o, ctx->cap_o_h, *ow))) return rc;
    if ((rc = upload(ctx, ctx->cap_o_b, *ob, false))) return rc;
    if ((rc = up2(ctx, ctx->cap_f0, ctx->cap_f0_h, *f0w))) return rc;
    if ((rc = upload(ctx, ctx->cap_f0_b, *f0b, false))) return rc;
    if ((rc = up2(ctx, ctx->cap_f3, ctx->cap_f3_h, *f3w))) return rc;
    if ((rc = upload(ctx, ctx->cap_f3_b, *f3b, false))) return rc;
    if ((rc = upload(ctx, ctx->cap_ng, *ng, false))) return rc;
    if ((rc = upload(ctx, ctx->cap_nb, *nb, false))) return rc;
    if (E == 192) {  // the bf16 tail runs on mlp_rows_kernel's CAP form
      if ((rc = upload(ctx, ctx->cap_f0_p, pack_mlp1_perm(*f0w, E, 2 * E), true))) return rc;
      if ((rc = upload(ctx, ctx->cap_f3_p, pack_mlp2_perm(*f3w, E, 2 * E), true))) return rc;
      std::vector<float> v;  // [bo | b0 | g | b + b3]
      for (const std::vector<float>* part : {ob, f0b, ng}) v.insert(v.end(), part->begin(), part->end());
      for (int e = 0; e < E; ++e) v.push_back((*nb)[e] + (*f3b)[e]);
      if ((rc = upload(ctx, ctx->cap_vecs, v, false))) return rc;
    }
  }
  if (d.mixer_type == MMPFN_MIXER_MOE) {
    const int ne = d.mgm_heads;
    std::vector<float> W1((size_t)ne * (D / 2) * D), B1((size_t)ne * (D / 2)), W2((size_t)ne * E * (D / 2)),
        B2((size_t)ne * E);
    for (int i = 0; i < ne; ++i) {
      const std::string p = "moe.experts." + std::to_string(i) + ".";
      GETW(g, p + "0.weight", (size_t)D);
      GETW(b, p + "0.bias", (size_t)D);
      GETW(w1, p + "1.weight", (size_t)(D / 2) * D);
      GETW(b1, p + "1.bias", (size_t)D / 2);
      GETW(w2, p + "4.weight", (size_t)E * (D / 2));
      GETW(b2, p + "4.bias", (size_t)E);
      std::vector<float> w = *w1, c = *b1;
      fold_ln(w, c, g->data(), b->data(), D / 2, D);
      std::copy(w.begin(), w.end(), W1.begin() + (size_t)i * (D / 2) * D);
      std::copy(c.begin(), c.end(), B1.begin() + (size_t)i * (D / 2));
      std::copy(w2->begin(), w2->end(), W2.begin() + (size_t)i * E * (D / 2));
      std::copy(b2->begin(), b2->end(), B2.begin() + (size_t)i * E);
    }
    GETW(gw, "moe.gate.weight", (size_t)ne * D);
    GETW(gb, "moe.gate.bias", (size_t)ne);
    if ((rc = up2(ctx, ctx->moe_w1, ctx->moe_w1_h, W1))) return rc;
    if ((rc = upload(ctx, ctx->moe_b1, B1, false))) return rc;
    if ((rc = up2(ctx, ctx->moe_w2, ctx->moe_w2_h, W2))) return rc;
    if ((rc = upload(ctx, ctx->moe_b2, B2, false))) return rc;
    if ((rc = upload(ctx, ctx->moe_gw, *gw, false))) return rc;
    if ((rc = upload(ctx, ctx->moe_gb, *gb, false))) return rc;
  }
  HIPCHK(hipDeviceSynchronize());
  return MMPFN_OK;
}

// weight operand of launch_gemm in a precision mode: bf16 copy, fp32 copy (PREC_F32_MFMA), or the
// hi | lo planes of the parity mode with the offset of the lo plane
void setw(const mmpfn_ctx* ctx, GemmArgs& a, const DevBuf& f, const DevBuf& h, int prec) {
  a.w_lo_off = 0;
  if (prec == PREC_BF16) {
    a.W = h.p;
  } else if (prec == PREC_F32) {
    const auto it = ctx->split.find(f.p);
    a.W = it == ctx->split.end() ? nullptr : it->second.p;
    a.w_lo_off = it == ctx->split.end() ? 0 : (int64_t)it->second.n;
  } else {
    a.W = f.p;
  }
}

// parity-mode row-resident projections (rowgemm3.hip): E = 192 = 6 heads of 32, split weights present
bool proj3_ok(const mmpfn_ctx* ctx, int prec) {
  return prec == PREC_F32 && ctx->d.emsize == 192 && ctx->d.nhead == 6;
}
Proj3Set p3set(const mmpfn_ctx* ctx, const DevBuf& f, const float* A, int64_t rdiv, int64_t rmul, int64_t rmul2,
               int64_t roff, int64_t M, int N) {
  const auto it = ctx->split.find(f.p);
  Proj3Set s{A, rdiv, rmul, rmul2, roff, nullptr, 0, (int)M, N};
  if (it != ctx->split.end()) s.W = it->second.p, s.w_lo = (int64_t)it->second.n;
  return s;
}
hipError_t p3_resln(const mmpfn_ctx* ctx, const DevBuf& f, const void* O, int64_t M, float* X, hipStream_t st) {
  const Proj3Set s = p3set(ctx, f, (const float*)O, 1, 1, 0, 0, M, 192);
  return launch_proj3_resln(s.A, s.W, s.w_lo, M, X, ctx->d.ln_eps, st);
}

GemmArgs gargs() {
  GemmArgs a;
  std::memset(&a, 0, sizeof(a));
  a.a_rdiv = 1ll << 62;
  a.a_rmul = 0;
  a.a_rmul2 = 1;
  a.rdiv2 = 1ll << 62;
  a.ln_eps = 1e-5f;
  return a;
}

#define RC(expr)                 \
  do {                           \
    int rc_ = (expr);            \
    if (rc_ != MMPFN_OK) return rc_; \
  } while (0)

// whether PREC_F16's layer kernels take this model / table: E = 192 in 6 heads and at most 64 tokens per row
// (T < 0: a row-wise sublayer, no token limit).  Everything else runs PREC_BF16 -- the forward (embed) and the
// per-sublayer taps (state_tap) apply the same rule.
#ifndef MMPFN_F16_QK_BF16
#define MMPFN_F16_QK_BF16 1  // PREC_F16's item Q / K in bf16 (0: fp16, S on the f16 MFMA; a diagnostics variant)
#endif

inline bool f16_fits(const mmpfn_model_desc& d, int T) { return d.emsize == 192 && d.nhead == 6 && T <= 64; }

// member m (of M, all of the geometry set by member 0) -> X[m] = embedded input [T][S][E]
int embed(mmpfn_ctx* ctx, const float* x, int S, int F, const float* tokens, int C, const float* y, int N,
          const float* uniq, int U, const float* pos_rand, int prec, int m = 0, int M = 1) {
  const mmpfn_model_desc& d = ctx->d;
  if (!ctx->finalized) return fail(ctx, MMPFN_ERR_STATE, "weights not finalised");
  if (S <= 0 || N <= 0 || N > S || (x && F <= 0) || C < 0 || U <= 0)
    return fail(ctx, MMPFN_ERR_INVALID, "bad forward geometry");
  if (!x && C == 0) return fail(ctx, MMPFN_ERR_INVALID, "no input tokens");
  if (!prec_ok(prec)) return fail(ctx, MMPFN_ERR_INVALID, "bad precision");
  const int f8 = f8_of(prec);
  prec = base_prec(prec);
  const int E = d.emsize, fpg = d.features_per_group;
  const int G = x ? (F + fpg - 1) / fpg : 0;
  const int T = G + C + 1;
  // PREC_F16's layer kernels hold a row's tokens as up to four 16-token tiles; wider tables run PREC_BF16
  if (prec == PREC_F16 && !f16_fits(d, T)) prec = PREC_BF16;
  const int Npad = (N + 63) / 64 * 64;
  const size_t R = (size_t)S * T;
  hipStream_t st = ctx->stream;
  int* flag;
  if (m == 0) {
    ctx->S = S, ctx->T = T, ctx->N = N, ctx->G = G, ctx->C = C, ctx->Npad = Npad, ctx->prec = prec, ctx->M = M;
    ctx->f8 = f8;
    RC(ensure(ctx, ctx->ws_X, (size_t)M * R * E * 4));
    RC(ensure(ctx, ctx->ws_O, (size_t)M * R * E * 4));
    const size_t Tpad = (T + 63) / 64 * 64;
    const size_t big = std::max(R * E + (size_t)2 * S * Tpad * E, (size_t)M * (R * E + (size_t)2 * T * Npad * E)) * 4;
    RC(ensure(ctx, ctx->ws_big, big));
    RC(ensure(ctx, ctx->ws_pe, (size_t)(G + C + 1) * E * 4));
    RC(ensure(ctx, ctx->ws_slots, (size_t)(G + 1) * fpg * sizeof(SlotParams)));
    RC(ensure(ctx, ctx->ws_scr, 256));
    RC(ensure_flag(ctx, ctx->ws_flag, st));
    flag = (int*)ctx->ws_flag.p;
    HIPCHK(launch_pos_emb(pos_rand, G + C, (const float*)ctx->pe_w.p, (const float*)ctx->pe_b.p,
                          (float*)ctx->ws_pe.p, E, st));
  } else {
    if (S != ctx->S || T != ctx->T || N != ctx->N || G != ctx->G || C != ctx->C || prec != ctx->prec || f8 != ctx->f8 ||
        m >= ctx->M)
      return fail(ctx, MMPFN_ERR_INVALID, "batched members must share S, N, F, C and precision");
    flag = (int*)ctx->ws_flag.p;
  }
  // the encoders write the state dtype directly (fp16 in PREC_F16)
  const bool h = prec == PREC_F16;
  void* X = (char*)ctx->ws_X.p + (size_t)m * R * E * (h ? 2 : 4);
  HIPCHK(launch_encode_stats(x, S, F, N, G, fpg, d.outlier_sigma, (SlotParams*)ctx->ws_slots.p, y, N,
                             (float*)ctx->ws_scr.p, st));
  HIPCHK(launch_assemble(x, S, F, G, fpg, d.encoder_features, (const SlotParams*)ctx->ws_slots.p,
                         (const float*)ctx->enc_w.p, (const float*)ctx->ws_pe.p, tokens, C, y, N, uniq, U,
                         (const float*)ctx->y_w.p, (const float*)ctx->y_b.p, (const float*)ctx->ws_scr.p, X, h, E, flag,
                         st));
  ctx->embedded = true;
  return MMPFN_OK;
}

// test rows against a train-KV cache: every row of the state is a test row (N = 0), the encoders
// apply the cached train statistics (transformer.py:779-784 use_cached_embeddings; encoders.py
// steps with cache_trainset_representation)
int embed_cached(mmpfn_ctx* ctx, const mmpfn_cache* cc, const float* x, int S, int F, const float* tokens, int C,
                 int prec) {
  const mmpfn_model_desc& d = ctx->d;
  if (!ctx->finalized) return fail(ctx, MMPFN_ERR_STATE, "weights not finalised");
  if (S <= 0 || F != cc->F || C != cc->C || prec != cc->prec || (F > 0 && !x) || (C > 0 && !tokens))
    return fail(ctx, MMPFN_ERR_INVALID, "test rows must match the cache's features, tokens and precision");
  const int E = d.emsize, fpg = d.features_per_group, G = cc->G, T = cc->T;
  const size_t R = (size_t)S * T;
  hipStream_t st = ctx->stream;
  ctx->S = S, ctx->T = T, ctx->N = 0, ctx->G = G, ctx->C = C, ctx->Npad = 0, ctx->prec = prec, ctx->M = 1;
  const bool h = prec == PREC_F16;
  ctx->f8 = 0;  // the cache keeps bf16 V^T: its test rows run the bf16 P.V
  RC(ensure(ctx, ctx->ws_X, R * E * 4));
  RC(ensure(ctx, ctx->ws_O, R * E * 4));
  const size_t Tpad = (T + 63) / 64 * 64;
  RC(ensure(ctx, ctx->ws_big, (R * E + (size_t)2 * S * Tpad * E) * 4));
  RC(ensure_flag(ctx, ctx->ws_flag, st));
  int* flag = (int*)ctx->ws_flag.p;
  HIPCHK(launch_assemble(x, S, F, G, fpg, d.encoder_features, (const SlotParams*)cc->slots.p,
                         (const float*)ctx->enc_w.p, (const float*)cc->pe.p, tokens, C, nullptr, 0,
                         (const float*)cc->uniq.p, cc->U, (const float*)ctx->y_w.p, (const float*)ctx->y_b.p,
                         (const float*)cc->ymean.p, ctx->ws_X.p, h, E, flag, st));
  ctx->embedded = true;
  return MMPFN_OK;
}

void cache_release(mmpfn_cache* cc) {
  for (DevBuf* b : {&cc->kv, &cc->slots, &cc->ymean, &cc->uniq, &cc->pe})
    if (b->p) (void)hipFree(b->p);
  delete cc;
}

// ---- attention between features (layer.py:332-339): X [M][T][S][E] <- LN(X + FeatAttn(X)), batch = row s
int feat_sublayer(mmpfn_ctx* ctx, const LayerW& L, void* Xv, int S, int T, int M, int prec) {
  const mmpfn_model_desc& d = ctx->d;
  const int E = d.emsize, H = d.nhead;
  const int64_t R = (int64_t)S * T;
  const bool bf = prec == PREC_BF16;
  const int eb = bf ? 2 : 4;
  hipStream_t st = ctx->stream;
  void* O = ctx->ws_O.p;
  unsigned char* big = (unsigned char*)ctx->ws_big.p;
  if (prec == PREC_F16) {  // fp16 state: the row-resident kernel only (embed keeps F16 to T <= 64)
    if (!L.feat_pack_f.p || T > 64) return fail(ctx, MMPFN_ERR_INVALID, "PREC_F16 needs E = 192, 6 heads, T <= 64");
    HIPCHK(launch_feat_rows(Xv, L.feat_pack_f.p, S, T, M, E, H, d.ln_eps, st, true));
    return MMPFN_OK;
  }
  float* Xall = (float*)Xv;
  if (bf && L.feat_pack_h.p && T <= 64) {
    // one wave per row (all M members' rows in one launch), the whole sublayer in registers (featrow.hip)
    HIPCHK(launch_feat_rows(Xall, L.feat_pack_h.p, S, T, M, E, H, d.ln_eps, st));
    return MMPFN_OK;
  }
  for (int m = 0; m < M; ++m) {  // member by member (the scratch holds one member)
    float* X = Xall + (size_t)m * R * E;
    if (bf && d.nhead * 32 == E && feat_block_rows(T) > 0) {
      HIPCHK(launch_feat_block(X, L.feat_qkv_h.p, L.feat_out_h.p, S, T, E, H, d.ln_eps, st));
      continue;
    }
    const int Tpad = (T + 63) / 64 * 64;
    void* Qf = big;
    void* Kf = big + (size_t)R * E * eb;
    void* Vf = (unsigned char*)Kf + (size_t)S * H * Tpad * 32 * eb;
    // logical rows m = s*T + t: A row t*S + s; scatter batch b = s, position t
    if (proj3_ok(ctx, prec)) {
      const Proj3Set ps = p3set(ctx, L.feat_qkv, X, T, 1, S, 0, R, 3 * E);
      HIPCHK(launch_proj3_qkv(&ps, 1, Qf, Kf, Vf, T, Tpad, H, st));
    } else {
      GemmArgs a = gargs();
      a.A = X, a.lda = E, a.a_rdiv = T, a.a_rmul = 1, a.a_rmul2 = S;
      setw(ctx, a, L.feat_qkv, L.feat_qkv_h, prec);
      a.M = (int)R, a.N = 3 * E, a.K = E;
      a.q = Qf, a.k = Kf, a.v = Vf, a.S = T, a.Npad = Tpad, a.T = T, a.H = H;
      HIPCHK(launch_gemm(a, prec, EPI_ITEM_QKV, true, !bf, 1, st));
    }
    AttnArgs f;
    f.q = Qf, f.k = Kf, f.vt = Vf, f.o = O;
    f.q_bstride = (int64_t)H * T * 32, f.q_hstride = (int64_t)T * 32;
    f.kv_bstride = (int64_t)H * Tpad * 32, f.kv_hstride = (int64_t)Tpad * 32, f.kpad = Tpad;
    f.o_bstride = 1, f.o_qstride = S;  // O[t][s]
    f.s0 = 0, f.nq = T, f.nk = T, f.kvh_fixed = -1, f.H = H;
    HIPCHK(launch_attn(f, S, prec, 1, st));
    if (proj3_ok(ctx, prec)) {
      HIPCHK(p3_resln(ctx, L.feat_out, O, R, X, st));
      continue;
    }
    GemmArgs b = gargs();
    b.A = O, b.lda = E, setw(ctx, b, L.feat_out, L.feat_out_h, prec);
    b.M = (int)R, b.N = E, b.K = E, b.X = X, b.ln_eps = d.ln_eps;
    HIPCHK(launch_gemm(b, prec, EPI_RES_LN, !bf, true, 1, st));
  }
  return MMPFN_OK;
}

// ---- attention between items (layer.py:341-379) of layer l; rows of all members: logical row
//      (member*T + t)*N + n -> memory row (member*T + t)*S + n, attention batch member*T + t.
//      fuse_out: the out-projection + residual + LN is left to the MLP kernel's prologue (the
//      attention output stays in ws_O); otherwise X <- LN(X + O Wout^T) here.
int item_sublayer(mmpfn_ctx* ctx, int l, void* Xv, int S, int T, int N, int Npad, int M, int prec,
                  bool fuse_out, int f8 = 0) {
  const mmpfn_model_desc& d = ctx->d;
  const LayerW& L = ctx->layers[l];
  const int E = d.emsize, H = d.nhead, Q = S - N;
  const int64_t RM = (int64_t)S * T * M;  // tokens of the batch
  const int TM = T * M;                   // token columns of the batch (attention batches)
  float* Xall = (float*)Xv;
  // PREC_F16 runs the bf16 mode's kernels in their F16 forms (fp16 X and O; bf16 Q, K (qkb) and V^T: the
  // attention's MFMAs all bf16)
  const bool h16 = prec == PREC_F16, qkb = h16 && MMPFN_F16_QK_BF16;
  if (h16 && E != 192) return fail(ctx, MMPFN_ERR_INVALID, "PREC_F16 needs E = 192");
  if (h16) prec = PREC_BF16;
  const bool bf = prec == PREC_BF16;
  const int eb = bf ? 2 : 4;
  hipStream_t st = ctx->stream;
  void* O = ctx->ws_O.p;
  unsigned char* big = (unsigned char*)ctx->ws_big.p;
  void* Qi = big;
  void* Ki = big + (size_t)RM * E * eb;
  void* Vi = (unsigned char*)Ki + (size_t)TM * H * Npad * 32 * eb;
  if (ctx->cache_in) {  // every row is a test row: Q only, against the cached train K/V of head 0
    const mmpfn_cache* cc = ctx->cache_in;
    const size_t kvl = (size_t)T * cc->Npad * 32 * eb;
    const unsigned char* Kc = (const unsigned char*)cc->kv.p + (size_t)l * 2 * kvl;
    const unsigned char* Vc = Kc + kvl;
    if (bf && E == 192) {
      HIPCHK(launch_rowgemm_qkv(Xv, S, S, 1, 0, h16 ? L.item_qtest_f.p : L.item_qtest_h.p, TM * S, E, Qi, Ki, Vi, S,
                                Npad, H, st, h16, qkb));
    } else if (proj3_ok(ctx, prec)) {
      const Proj3Set ps = p3set(ctx, L.item_qtest, Xall, S, S, 1, 0, (int64_t)TM * S, E);
      HIPCHK(launch_proj3_qkv(&ps, 1, Qi, Ki, Vi, S, Npad, H, st));
    } else {
      GemmArgs c = gargs();
      c.A = Xall, c.lda = E, c.a_rdiv = S, c.a_rmul = S, c.a_roff = 0;
      setw(ctx, c, L.item_qtest, L.item_qtest_h, prec);
      c.M = TM * S, c.N = E, c.K = E;
      c.q = Qi, c.k = Ki, c.v = Vi, c.S = S, c.Npad = Npad, c.T = TM, c.H = H;
      HIPCHK(launch_gemm(c, prec, EPI_ITEM_QKV, true, !bf, 1, st));
    }
    const int64_t cstride = (int64_t)cc->Npad * 32;
    if (bf)
      HIPCHK(launch_attn_layer(Qi, Kc, Vc, O, S, TM, H, cc->Npad, cc->N, 0, 0, 0, S, 0, st, cstride, true, nullptr, 0,
                               h16 && !qkb, h16));
    else
      HIPCHK(launch_attn_item(Qi, Kc, Vc, O, S, TM, H, cc->Npad, 0, S, cc->N, 0, prec, st, cstride));
  } else {
    if (bf && E == 192) {  // row-resident projections straight into the attention layouts
      // train rows q|k|v and test rows q in one launch (test-row blocks last)
      HIPCHK(launch_rowgemm_qkv_pair(Xv, N, 0, h16 ? L.item_qkv_f.p : L.item_qkv_h.p, TM * N, 3 * E, Q, N,
                                     h16 ? L.item_qtest_f.p : L.item_qtest_h.p, TM * Q, E, S, Qi, Ki, Vi, S, Npad, H, st,
                                     h16, qkb));
    } else if (proj3_ok(ctx, prec)) {  // train rows q|k|v and test rows q in one launch
      const Proj3Set ps[2] = {p3set(ctx, L.item_qkv, Xall, N, S, 1, 0, (int64_t)TM * N, 3 * E),
                              p3set(ctx, L.item_qtest, Xall, Q > 0 ? Q : 1, S, 1, N, (int64_t)TM * Q, E)};
      HIPCHK(launch_proj3_qkv(ps, 2, Qi, Ki, Vi, S, Npad, H, st));
    } else {
      GemmArgs a = gargs();
      a.A = Xall, a.lda = E, a.a_rdiv = N, a.a_rmul = S, a.a_roff = 0;
      setw(ctx, a, L.item_qkv, L.item_qkv_h, prec);
      a.M = TM * N, a.N = 3 * E, a.K = E;
      a.q = Qi, a.k = Ki, a.v = Vi, a.S = S, a.Npad = Npad, a.T = TM, a.H = H;
      HIPCHK(launch_gemm(a, prec, EPI_ITEM_QKV, true, !bf, 1, st));
      if (Q > 0) {
        GemmArgs c = a;
        c.a_rdiv = Q, c.a_roff = N;
        setw(ctx, c, L.item_qtest, L.item_qtest_h, prec);
        c.M = TM * Q, c.N = E;
        HIPCHK(launch_gemm(c, prec, EPI_ITEM_QKV, true, !bf, 1, st));
      }
    }
    if (ctx->cache_out) {  // keep head 0's K / V^T of every column (the test rows' KV, layer.py:344-358)
      mmpfn_cache* cc = ctx->cache_out;
      const size_t blk = (size_t)Npad * 32 * eb, kvl = (size_t)T * blk;
      unsigned char* Kc = (unsigned char*)cc->kv.p + (size_t)l * 2 * kvl;
      HIPCHK(hipMemcpy2DAsync(Kc, blk, Ki, (size_t)H * blk, blk, T, hipMemcpyDeviceToDevice, st));
      HIPCHK(hipMemcpy2DAsync(Kc + kvl, blk, Vi, (size_t)H * blk, blk, T, hipMemcpyDeviceToDevice, st));
    }
    if (bf) {  // train rows (own heads) and test rows (head-0 K/V, MQA) in one launch
      hipEvent_t* ev = nullptr;
      if (ctx->kt_on) {
        if (ctx->kt_used + 2 > ctx->kt_pool.size()) {
          for (int i = 0; i < 64; ++i) {
            hipEvent_t e;
            HIPCHK(hipEventCreate(&e));
            ctx->kt_pool.push_back(e);
          }
        }
        ev = &ctx->kt_pool[ctx->kt_used];
        ctx->kt_used += 2;
        ctx->kt_flops += 4.0 * TM * (double)(N + Q) * N * E;
      }
      void* V8 = nullptr;
      if (f8) {  // e4m3 V^T after the bf16 one (ws_big holds twice the bf16 Q / K / V^T bytes)
        V8 = (unsigned char*)Vi + (size_t)TM * H * Npad * 32 * eb;
        HIPCHK(launch_vt_fp8(Vi, V8, (int64_t)TM * H * Npad * 32, st));
      }
      if (ev) HIPCHK(hipEventRecord(ev[0], st));
      HIPCHK(launch_attn_layer(Qi, Ki, Vi, O, S, TM, H, Npad, N, 0, N, N, Q, 0, st, 0, true, V8, f8, h16 && !qkb, h16));
      if (ev) HIPCHK(hipEventRecord(ev[1], st));
    } else if (prec == PREC_F32) {  // parity mode: split-bf16 products, train and test rows in one launch
      HIPCHK(launch_attn_item3(Qi, Ki, Vi, O, S, TM, H, Npad, N, 0, N, N, Q, 0, st));
    } else {
      HIPCHK(launch_attn_item(Qi, Ki, Vi, O, S, TM, H, Npad, 0, N, N, -1, prec, st));
      if (Q > 0) HIPCHK(launch_attn_item(Qi, Ki, Vi, O, S, TM, H, Npad, N, Q, N, 0, prec, st));
    }
  }
  if (fuse_out) return MMPFN_OK;
  if (bf && E == 192) {
    HIPCHK(launch_rowgemm_resln(O, h16 ? L.item_out_f.p : L.item_out_h.p, RM, Xv, d.ln_eps, st, h16));
  } else if (proj3_ok(ctx, prec)) {
    HIPCHK(p3_resln(ctx, L.item_out, O, RM, Xall, st));
  } else {
    GemmArgs b = gargs();
    b.A = O, b.lda = E, setw(ctx, b, L.item_out, L.item_out_h, prec);
    b.M = (int)RM, b.N = E, b.K = E, b.X = Xall, b.ln_eps = d.ln_eps;
    HIPCHK(launch_gemm(b, prec, EPI_RES_LN, !bf, true, 1, st));
  }
  return MMPFN_OK;
}

// the bf16 MLP kernel runs the item-attention out-projection as its prologue
bool mlp_fuses_out(const mmpfn_model_desc& d, int prec) {
  return prec16(prec) && d.emsize == 192 && d.nhid % 32 == 0;
}

// ---- MLP (mlp.py:93-104) + residual + LN over RM tokens; O non-null: the fused out-projection first
int mlp_sublayer(mmpfn_ctx* ctx, const LayerW& L, void* Xv, int64_t RM, int prec, const void* O) {
  const mmpfn_model_desc& d = ctx->d;
  float* Xall = (float*)Xv;
  if (prec == PREC_F16) {  // fp16 copies: W1 natural, W2 / Wout rows in f16_row_perm order
    if (!mlp_fuses_out(d, prec) || !L.mlp1_f.p) return fail(ctx, MMPFN_ERR_INVALID, "PREC_F16 needs E = 192");
    HIPCHK(launch_mlp_rows(Xv, L.mlp1_f.p, L.mlp2_f.p, RM, d.emsize, d.nhid, d.ln_eps, ctx->stream, O,
                           O ? L.item_out_f.p : nullptr, true));
  } else if (mlp_fuses_out(d, prec)) {  // W1 / W2 bf16 copies in mlp_rows_kernel's K orders
    HIPCHK(launch_mlp_rows(Xall, L.mlp1_h.p, L.mlp2_h.p, RM, d.emsize, d.nhid, d.ln_eps, ctx->stream, O,
                           O ? L.item_out_h.p : nullptr));
  } else if (prec == PREC_F32) {  // parity mode: mlp_x3_kernel on split-bf16 products (W1 / W2 hi | lo planes)
    const auto w1 = ctx->split.find(L.mlp1.p), w2 = ctx->split.find(L.mlp2_h.p);  // W1 natural, W2 permuted
    if (w1 == ctx->split.end() || w2 == ctx->split.end()) return fail(ctx, MMPFN_ERR_STATE, "no split MLP weights");
    HIPCHK(launch_mlp_fused(Xall, w1->second.p, w2->second.p, RM, d.emsize, d.nhid, d.ln_eps, PREC_F32, ctx->stream));
  } else {
    HIPCHK(launch_mlp_fused(Xall, L.mlp1.p, L.mlp2.p, RM, d.emsize, d.nhid, d.ln_eps, PREC_F32_MFMA, ctx->stream));
  }
  return MMPFN_OK;
}

int run_layer(mmpfn_ctx* ctx, int l) {
  const LayerW& L = ctx->layers[l];
  const int S = ctx->S, T = ctx->T, N = ctx->N, Npad = ctx->Npad, prec = ctx->prec, M = ctx->M;
  void* Xall = ctx->ws_X.p;
  const bool fuse = mlp_fuses_out(ctx->d, prec);
  RC(feat_sublayer(ctx, L, Xall, S, T, M, prec));
  RC(item_sublayer(ctx, l, Xall, S, T, N, Npad, M, prec, fuse, ctx->f8));
  return mlp_sublayer(ctx, L, Xall, (int64_t)S * T * M, prec, fuse ? ctx->ws_O.p : nullptr);
}

// workspace of the selected lane for a per-sublayer tap on a caller-provided state of S x T tokens
int tap_workspace(mmpfn_ctx* ctx, int S, int T, int Npad) {
  const int E = ctx->d.emsize;
  const size_t R = (size_t)S * T;
  const size_t Tpad = (T + 63) / 64 * 64;
  RC(ensure(ctx, ctx->ws_O, R * E * 4));
  RC(ensure(ctx, ctx->ws_big, std::max(R * E + 2 * S * Tpad * E, R * E + (size_t)2 * T * Npad * E) * 4));
  return MMPFN_OK;
}

// decoder over the test rows of M batched members (logits [M][Q][n_out]); the tile partials go
// through the attention-output workspace, free once the last layer has run
int decode(mmpfn_ctx* ctx, float* logits, int M = 1) {
  const mmpfn_model_desc& d = ctx->d;
  const int E = d.emsize, S = ctx->S, T = ctx->T, N = ctx->N, Q = S - N;
  const size_t off = ((size_t)(T - 1) * S + N) * E;
  const float* Xl = (const float*)ctx->ws_X.p + off;
  int64_t xm = (int64_t)S * T * E;
  if (prec16(ctx->prec) && ctx->dec_w1_h.p) {  // the state as it is (fp32 / fp16) into 16-bit MFMA operands
    const bool h = ctx->prec == PREC_F16;
    const void* X = (const char*)ctx->ws_X.p + off * (h ? 2 : 4);
    HIPCHK(launch_decoder_mfma(X, h, Q, h ? ctx->dec_w1_f.p : ctx->dec_w1_h.p, (const float*)ctx->dec_b1.p, d.nhid,
                               h ? ctx->dec_w2p_f.p : ctx->dec_w2p_h.p, (const float*)ctx->dec_b2.p, d.n_out, logits, E,
                               ctx->stream, M, xm, (int64_t)Q * d.n_out));
    return MMPFN_OK;
  }
  if (ctx->prec == PREC_F16) {  // the target token's test rows of every member to fp32 (the big workspace is free)
    RC(ensure(ctx, ctx->ws_big, (size_t)M * Q * E * 4));
    HIPCHK(launch_f16_to_f32((const uint16_t*)ctx->ws_X.p + off, xm, (float*)ctx->ws_big.p, (int64_t)Q * E,
                             (int64_t)Q * E, M, ctx->stream));
    Xl = (const float*)ctx->ws_big.p, xm = (int64_t)Q * E;
  }
  RC(ensure(ctx, ctx->ws_O, (size_t)M * (d.nhid / 32 + 1) * Q * d.n_out * sizeof(float)));
  HIPCHK(launch_decoder(Xl, Q, (const float*)ctx->dec_w1.p, (const float*)ctx->dec_b1.p, d.nhid,
                        (const float*)ctx->dec_w2.p, (const float*)ctx->dec_b2.p, d.n_out, logits, E, ctx->stream, M,
                        xm, (int64_t)Q * d.n_out, (float*)ctx->ws_O.p));
  return MMPFN_OK;
}

// MGM head bank (transformer.py:33-57): image [S][n_mod][D] -> tokens [S][mgm*n_mod][E] (head-major)
// tok16: the tokens in 16-bit (the MGM+CAP chain's intermediate; bf16, or fp16 under PREC_F16; E = 192 only).
// PREC_F16 runs the head bank on fp16 operands (LN output, GLU hidden, weights) where the big-tile kernels take
// the shape, else in the bf16 mode: fp16's 3 extra mantissa bits cut the mixer's share of the logits error ~7x
// (DESIGN 3, 6), and the reference's own fp16 autocast runs these linears in fp16.
bool mgm_f16(const mmpfn_ctx* ctx) { return ctx->mgm_w1_f.p != nullptr && mgm_f16_shape(ctx->d); }

int mixer_mgm(mmpfn_ctx* ctx, const float* image, int S, int n_mod, void* mtok, int prec, bool tok16 = false) {
  const mmpfn_model_desc& d = ctx->d;
  const int E = d.emsize, D = d.nhid;
  if (prec == PREC_F16 && !mgm_f16(ctx)) prec = PREC_BF16;
  const bool h = prec == PREC_F16, bf = prec == PREC_BF16 || h;
  const int eb = bf ? 2 : 4;
  hipStream_t st = ctx->stream;
  const int64_t rows = (int64_t)S * n_mod;
  const int mg = d.mgm_heads, M = mg * n_mod;
  RC(ensure(ctx, ctx->mx[0], (size_t)rows * D * eb));             // normalised image
  RC(ensure(ctx, ctx->mx[1], (size_t)rows * mg * (D / 2) * eb));  // GLU output
  HIPCHK(launch_layernorm_rows(image, rows, D, 1e-5f, ctx->mx[0].p, !bf, nullptr, nullptr, st, h));
  GemmArgs a = gargs();
  a.A = ctx->mx[0].p, a.lda = D, setw(ctx, a, ctx->mgm_w1, ctx->mgm_w1_h, prec), a.bias = (const float*)ctx->mgm_b1.p;
  a.M = (int)rows, a.N = mg * D, a.K = D, a.C = ctx->mx[1].p, a.ldc = (int64_t)mg * (D / 2);
  const bool big2 = bf && E == 192 && (D / 2) % 32 == 0;  // the big-tile down-projection (16-bit tokens possible)
  if (bf && (mg * D) % 256 == 0 && D % 64 == 0)
    HIPCHK(launch_gemm_glu_big(ctx->mx[0].p, h ? ctx->mgm_w1_f.p : a.W, a.bias, ctx->mx[1].p, (int)rows, mg * D, D,
                               st, h));
  else
    HIPCHK(launch_gemm(a, prec, EPI_GLU, !bf, !bf, 1, st));
  GemmArgs b = gargs();
  b.A = ctx->mx[1].p, b.lda = (int64_t)mg * (D / 2), b.a_zstride = D / 2;
  setw(ctx, b, ctx->mgm_w2, ctx->mgm_w2_h, prec), b.w_zstride = (int64_t)E * (D / 2);
  b.bias = (const float*)ctx->mgm_b2.p, b.b_zstride = E;
  b.M = (int)rows, b.N = E, b.K = D / 2;
  b.C = mtok, b.ldc = E, b.rdiv2 = n_mod, b.rmul2 = M, b.zmul = n_mod;
  if (tok16 && !big2) return fail(ctx, MMPFN_ERR_INVALID, "16-bit MGM tokens");
  if (big2)
    HIPCHK(launch_gemm_remap_big(ctx->mx[1].p, (int64_t)mg * (D / 2), h ? ctx->mgm_w2_f.p : ctx->mgm_w2_h.p,
                                 (const float*)ctx->mgm_b2.p, mtok, tok16, (int)rows, D / 2, mg, n_mod, E, st, h));
  else
    HIPCHK(launch_gemm(b, prec, EPI_REMAP, !bf, true, mg, st));
  return MMPFN_OK;
}

// CrossAttentionPooler (transformer.py:60-88): MGM tokens [S][M][E] -> tokens [S][cap][E]
// mtok fp32, or 16-bit (in16: from mixer_mgm's bf16 form, fp16 under PREC_F16); PREC_F16 runs the pooler in the
// bf16 mode from the row pass on (its K|V, attention and tail stay bf16)
int mixer_cap(mmpfn_ctx* ctx, const void* mtok, int S, int M, float* tokens, int prec, bool in16 = false) {
  const mmpfn_model_desc& d = ctx->d;
  const int E = d.emsize;
  const bool in_f16 = in16 && prec == PREC_F16, in_bf16 = in16 && !in_f16;
  if (prec == PREC_F16) prec = PREC_BF16;
  const bool bf = prec == PREC_BF16;
  const int eb = bf ? 2 : 4;
  hipStream_t st = ctx->stream;
  const int cap = d.cap_heads;
  const int64_t srows = (int64_t)S * M;
  RC(ensure(ctx, ctx->mx[3], (size_t)srows * E * eb));        // k_norm(src) (affine folded)
  RC(ensure(ctx, ctx->mx[4], (size_t)srows * 2 * E * eb));    // K|V
  RC(ensure(ctx, ctx->mx[5], (size_t)S * cap * E * 4));       // attention out (heads concat)
  RC(ensure(ctx, ctx->mx[6], (size_t)S * cap * E * 4));       // out_proj
  RC(ensure(ctx, ctx->mx[7], (size_t)S * cap * 2 * E * 4));   // ffn hidden (+ ffn out after)
  // bf16, E = 192, 24 heads over M % 32 == 0 tokens: K [S*M][E] and V^T [S][E][M] for the MFMA attention
  const bool mf = bf && E == 192 && cap == 24 && M % 32 == 0 && M <= 128 && ctx->cap_vecs.p;
  void* vt = (char*)ctx->mx[4].p + (size_t)srows * E * 2;
  if (bf && E == 192) {  // k_norm + K|V projection in one row pass (normalised rows stay in registers)
    HIPCHK(launch_rowgemm_ln_store(mtok, in_bf16, ctx->cap_kv_h.p, (const float*)ctx->cap_kv_b.p, ctx->mx[4].p, srows,
                                   2 * E, 1e-5f, true, st, mf ? vt : nullptr, E, M, in_f16));
  } else {
    HIPCHK(launch_layernorm_rows((const float*)mtok, srows, E, 1e-5f, ctx->mx[3].p, !bf, nullptr, nullptr, st));
    GemmArgs c = gargs();
    c.A = ctx->mx[3].p, c.lda = E, setw(ctx, c, ctx->cap_kv, ctx->cap_kv_h, prec), c.bias = (const float*)ctx->cap_kv_b.p;
    c.M = (int)srows, c.N = 2 * E, c.K = E, c.C = ctx->mx[4].p, c.ldc = 2 * E;
    HIPCHK(launch_gemm(c, prec, EPI_STORE, !bf, !bf, 1, st));
  }
  const int64_t crow = (int64_t)S * cap;
  if (bf && E == 192 && ctx->cap_vecs.p) {  // attention out in bf16, then the whole tail in one row-resident pass
    if (mf)
      HIPCHK(launch_cap_attention_mfma((const float*)ctx->cap_qp.p, ctx->mx[4].p, vt, ctx->mx[5].p, S, M, cap, E, st));
    else
      HIPCHK(launch_cap_attention((const float*)ctx->cap_qp.p, ctx->mx[4].p, false, ctx->mx[5].p, true, S, M, cap, E,
                                  st));
    HIPCHK(launch_cap_tail(ctx->mx[5].p, ctx->cap_o_h.p, ctx->cap_f0_p.p, ctx->cap_f3_p.p,
                           (const float*)ctx->cap_vecs.p, tokens, crow, E, 1e-5f, st));
    return MMPFN_OK;
  }
  HIPCHK(launch_cap_attention((const float*)ctx->cap_qp.p, ctx->mx[4].p, !bf, ctx->mx[5].p, false, S, M, cap, E, st));
  // projections run in fp32 A (tiny); bf16 weights in perf mode
  GemmArgs o = gargs();
  o.A = ctx->mx[5].p, o.lda = E, setw(ctx, o, ctx->cap_o, ctx->cap_o_h, prec), o.bias = (const float*)ctx->cap_o_b.p;
  o.M = (int)crow, o.N = E, o.K = E, o.C = ctx->mx[6].p, o.ldc = E;
  HIPCHK(launch_gemm(o, prec, EPI_STORE, true, true, 1, st));
  GemmArgs f0 = gargs();
  f0.A = ctx->mx[6].p, f0.lda = E, setw(ctx, f0, ctx->cap_f0, ctx->cap_f0_h, prec);
  f0.bias = (const float*)ctx->cap_f0_b.p, f0.act = ACT_GELU;
  f0.M = (int)crow, f0.N = 2 * E, f0.K = E, f0.C = ctx->mx[7].p, f0.ldc = 2 * E;
  HIPCHK(launch_gemm(f0, prec, EPI_STORE, true, true, 1, st));
  GemmArgs f3 = gargs();
  f3.A = ctx->mx[7].p, f3.lda = 2 * E, setw(ctx, f3, ctx->cap_f3, ctx->cap_f3_h, prec);
  f3.bias = (const float*)ctx->cap_f3_b.p;
  f3.M = (int)crow, f3.N = E, f3.K = 2 * E, f3.C = ctx->mx[5].p, f3.ldc = E;  // reuse mx5 for ffn out
  HIPCHK(launch_gemm(f3, prec, EPI_STORE, true, true, 1, st));
  HIPCHK(launch_ln_add((const float*)ctx->mx[6].p, (const float*)ctx->mx[5].p, (const float*)ctx->cap_ng.p,
                       (const float*)ctx->cap_nb.p, tokens, crow, E, 1e-5f, st));
  return MMPFN_OK;
}

int mixer(mmpfn_ctx* ctx, const float* image, int S, int n_mod, float* tokens, int prec) {
  const mmpfn_model_desc& d = ctx->d;
  const int E = d.emsize, D = d.nhid;
  if (d.mixer_type == MMPFN_MIXER_MGM) return mixer_mgm(ctx, image, S, n_mod, tokens, prec);
  if (d.mixer_type == MMPFN_MIXER_MGM_CAP) {
    const int M = d.mgm_heads * n_mod;
    RC(ensure(ctx, ctx->mx[2], (size_t)S * M * E * 4));
    if (prec == PREC_F16 && !mgm_f16(ctx)) prec = PREC_BF16;
    const bool b16 = prec == PREC_BF16 || prec == PREC_F16;
    const bool tb = b16 && E == 192 && (D / 2) % 32 == 0;  // 16-bit intermediate tokens (half the HBM bytes)
    RC(mixer_mgm(ctx, image, S, n_mod, ctx->mx[2].p, prec, tb));
    return mixer_cap(ctx, ctx->mx[2].p, S, M, tokens, prec, tb);
  }
  if (prec == PREC_F16) prec = PREC_BF16;  // the MoE mixer runs the bf16 mode
  const bool bf = prec == PREC_BF16;
  const int eb = bf ? 2 : 4;
  hipStream_t st = ctx->stream;
  if (d.mixer_type == MMPFN_MIXER_MOE) {
    const int ne = d.mgm_heads;
    RC(ensure(ctx, ctx->mx[0], (size_t)S * D * eb));
    RC(ensure(ctx, ctx->mx[1], (size_t)S * ne * (D / 2) * eb));
    RC(ensure(ctx, ctx->mx[2], (size_t)S * ne * 4));
    // modality 0 rows: image + s*n_mod*D  -> normalise with row stride n_mod*D
    // (ln kernel assumes contiguous rows; handle stride by normalising all rows when n_mod==1,
    //  else gather modality 0 first)
    const float* x0 = image;
    if (n_mod != 1) {
      RC(ensure(ctx, ctx->mx[3], (size_t)S * D * 4));
      HIPCHK(hipMemcpy2DAsync(ctx->mx[3].p, (size_t)D * 4, image, (size_t)n_mod * D * 4, (size_t)D * 4, S,
                              hipMemcpyDeviceToDevice, st));
      x0 = (const float*)ctx->mx[3].p;
    }
    HIPCHK(launch_layernorm_rows(x0, S, D, 1e-5f, ctx->mx[0].p, !bf, nullptr, nullptr, st));
    GemmArgs a = gargs();
    a.A = ctx->mx[0].p, a.lda = D, setw(ctx, a, ctx->moe_w1, ctx->moe_w1_h, prec), a.bias = (const float*)ctx->moe_b1.p;
    a.act = ACT_GELU, a.M = S, a.N = ne * (D / 2), a.K = D, a.C = ctx->mx[1].p, a.ldc = (int64_t)ne * (D / 2);
    HIPCHK(launch_gemm(a, prec, EPI_STORE, !bf, !bf, 1, st));
    GemmArgs b = gargs();
    b.A = ctx->mx[1].p, b.lda = (int64_t)ne * (D / 2), b.a_zstride = D / 2;
    setw(ctx, b, ctx->moe_w2, ctx->moe_w2_h, prec), b.w_zstride = (int64_t)E * (D / 2);
    b.bias = (const float*)ctx->moe_b2.p, b.b_zstride = E;
    b.M = S, b.N = E, b.K = D / 2, b.C = tokens, b.ldc = E, b.rdiv2 = 1, b.rmul2 = ne, b.zmul = 1;
    HIPCHK(launch_gemm(b, prec, EPI_REMAP, !bf, true, ne, st));
    HIPCHK(launch_gate_softmax(x0, D, S, D, (const float*)ctx->moe_gw.p, (const float*)ctx->moe_gb.p, ne,
                               (float*)ctx->mx[2].p, st));
    HIPCHK(launch_scale_tokens(tokens, (const float*)ctx->mx[2].p, S, ne, E, st));
    return MMPFN_OK;
  }
  return fail(ctx, MMPFN_ERR_INVALID, "model has no mixer");
}

// a tap on the caller's fp32 state: PREC_F16 runs it on an fp16 copy and converts the result back
// (T: the state's tokens per row, -1 for a row-wise sublayer; where f16_fits says no, the sublayer runs PREC_BF16,
// as the forward does)
template <typename F>
int state_tap(mmpfn_ctx* ctx, float* X, int64_t n, int precision, int T, F&& run) {
  int bp = base_prec(precision);
  if (bp == PREC_F16 && !f16_fits(ctx->d, T)) bp = PREC_BF16;
  if (bp != PREC_F16) return run((void*)X, bp);
  RC(ensure(ctx, ctx->tap_x16, (size_t)n * 2));
  HIPCHK(launch_f32_to_f16(X, 0, ctx->tap_x16.p, 0, n, 1, ctx->stream));
  RC(run(ctx->tap_x16.p, bp));
  HIPCHK(launch_f16_to_f32(ctx->tap_x16.p, 0, X, 0, n, 1, ctx->stream));
  return MMPFN_OK;
}

}  // namespace

// ===================================================================== C ABI
extern "C" {

const char* mmpfn_version(void) { return "mmpfn-hip 0.1 (gfx950)"; }

mmpfn_ctx* mmpfn_create(int device, void* stream) {
  if (hipSetDevice(device) != hipSuccess) return nullptr;
  mmpfn_ctx* c = new mmpfn_ctx();
  c->device = device;
  c->stream = (hipStream_t)stream;
  c->seen_streams.push_back(c->stream);
  return c;
}

void mmpfn_destroy(mmpfn_ctx* ctx) {
  if (!ctx) return;
  // teardown: errors here have no caller to report to
  (void)hipSetDevice(ctx->device);
  (void)hipStreamSynchronize(ctx->stream);
  (void)hipDeviceSynchronize();  // lanes may still be running on other streams
  for (hipEvent_t e : ctx->kt_pool) (void)hipEventDestroy(e);
  auto fr = [](DevBuf& b) {
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
  };
  for (auto& L : ctx->layers) {
    for (DevBuf* b : {&L.feat_qkv, &L.feat_out, &L.item_qkv, &L.item_qtest, &L.item_out, &L.mlp1, &L.mlp2,
                      &L.feat_qkv_h, &L.feat_out_h, &L.item_qkv_h, &L.item_qtest_h, &L.item_out_h, &L.mlp1_h,
                      &L.mlp2_h, &L.feat_pack_h, &L.feat_pack_f, &L.item_qkv_f, &L.item_qtest_f, &L.item_out_f,
                      &L.mlp1_f, &L.mlp2_f})
      fr(*b);
  }
  for (DevBuf* b : {&ctx->dec_w1_h, &ctx->dec_w1_f, &ctx->dec_w2p_h, &ctx->dec_w2p_f}) fr(*b);
  for (DevBuf* b : {&ctx->enc_w, &ctx->y_w, &ctx->y_b, &ctx->pe_w, &ctx->pe_b, &ctx->dec_w1, &ctx->dec_b1,
                    &ctx->dec_w2, &ctx->dec_b2, &ctx->mgm_w1, &ctx->mgm_w1_h, &ctx->mgm_b1, &ctx->mgm_w2,
                    &ctx->mgm_w2_h, &ctx->mgm_b2, &ctx->mgm_w1_f, &ctx->mgm_w2_f, &ctx->cap_qp, &ctx->cap_kv,
                    &ctx->cap_kv_h, &ctx->cap_kv_b,
                    &ctx->cap_o, &ctx->cap_o_h, &ctx->cap_o_b, &ctx->cap_f0, &ctx->cap_f0_h, &ctx->cap_f0_b,
                    &ctx->cap_f3, &ctx->cap_f3_h, &ctx->cap_f3_b, &ctx->cap_ng, &ctx->cap_nb, &ctx->cap_f0_p,
                    &ctx->cap_f3_p, &ctx->cap_vecs, &ctx->moe_w1, &ctx->moe_w1_h, &ctx->moe_b1, &ctx->moe_w2, &ctx->moe_w2_h, &ctx->moe_b2, &ctx->moe_gw,
                    &ctx->moe_gb, &ctx->ws_X, &ctx->ws_O, &ctx->ws_big, &ctx->ws_pe, &ctx->ws_slots, &ctx->ws_scr,
                    &ctx->ws_flag, &ctx->tap_v8, &ctx->tap_x16})
    fr(*b);
  for (auto& b : ctx->mx) fr(b);
  for (auto& kv : ctx->split) fr(kv.second);
  for (auto& L : ctx->lanes)
    for (DevBuf* b : {&L.ws_X, &L.ws_O, &L.ws_big, &L.ws_pe, &L.ws_slots, &L.ws_scr, &L.ws_flag}) fr(*b);
  delete ctx;
}

int mmpfn_select_lane(mmpfn_ctx* ctx, int lane) {
  if (!ctx || lane < 0 || lane >= MMPFN_MAX_LANES) return MMPFN_ERR_INVALID;
  if (lane == ctx->cur) return MMPFN_OK;
  if ((int)ctx->lanes.size() < MMPFN_MAX_LANES) ctx->lanes.resize(MMPFN_MAX_LANES);
  mmpfn_ctx::swap_lane(*ctx, ctx->lanes[ctx->cur]);   // park the selected lane
  mmpfn_ctx::swap_lane(*ctx, ctx->lanes[lane]);       // bring the requested one in
  ctx->cur = lane;
  return MMPFN_OK;
}

const char* mmpfn_last_error(const mmpfn_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int mmpfn_set_stream(mmpfn_ctx* ctx, void* stream) {
  if (!ctx) return MMPFN_ERR_INVALID;
  ctx->stream = (hipStream_t)stream;
  bool known = false;
  for (hipStream_t s : ctx->seen_streams) known |= s == ctx->stream;
  if (!known) ctx->seen_streams.push_back(ctx->stream);
  return MMPFN_OK;
}

int mmpfn_set_model(mmpfn_ctx* ctx, const mmpfn_model_desc* desc) {
  if (!ctx || !desc) return MMPFN_ERR_INVALID;
  const mmpfn_model_desc& d = *desc;
  if (d.emsize != 192 || d.nhead * 32 != d.emsize)
    return fail(ctx, MMPFN_ERR_INVALID, "engine is specialised for emsize 192 with head dim 32");
  if (d.nhid % 192 != 0 || d.nlayers <= 0 || d.features_per_group <= 0 || d.features_per_group > 8 ||
      d.encoder_features < d.features_per_group || d.encoder_features > 8 || d.n_out <= 0)
    return fail(ctx, MMPFN_ERR_INVALID, "unsupported model geometry");
  if (d.mixer_type == MMPFN_MIXER_MGM_CAP && (d.cap_heads <= 0 || d.emsize % d.cap_heads != 0))
    return fail(ctx, MMPFN_ERR_INVALID, "cap_heads must divide emsize");
  ctx->d = d;
  ctx->have_model = true;
  ctx->finalized = false;
  ctx->host.clear();
  return MMPFN_OK;
}

int mmpfn_load_weight(mmpfn_ctx* ctx, const char* name, const float* data, int64_t numel) {
  if (!ctx || !name || (!data && numel)) return MMPFN_ERR_INVALID;
  if (!ctx->have_model) return fail(ctx, MMPFN_ERR_STATE, "mmpfn_set_model first");
  ctx->host[name].assign(data, data + numel);
  ctx->finalized = false;
  return MMPFN_OK;
}

int mmpfn_finalize_weights(mmpfn_ctx* ctx) {
  if (!ctx) return MMPFN_ERR_INVALID;
  if (!ctx->have_model) return fail(ctx, MMPFN_ERR_STATE, "mmpfn_set_model first");
  HIPCHK(hipSetDevice(ctx->device));
  int rc = finalize(ctx);
  if (rc == MMPFN_OK) {
    ctx->finalized = true;
    ctx->host.clear();
  }
  return rc;
}

int mmpfn_mixer_tokens(const mmpfn_ctx* ctx, int n_mod) {
  if (!ctx) return MMPFN_ERR_INVALID;
  switch (ctx->d.mixer_type) {
    case MMPFN_MIXER_MGM: return ctx->d.mgm_heads * n_mod;
    case MMPFN_MIXER_MGM_CAP: return ctx->d.cap_heads;
    case MMPFN_MIXER_MOE: return ctx->d.mgm_heads;
  }
  return 0;
}

int mmpfn_mixer_forward(mmpfn_ctx* ctx, const float* image, int S, int n_mod, float* tokens, int precision) {
  if (!ctx || !image || !tokens || S <= 0 || n_mod <= 0) return MMPFN_ERR_INVALID;
  if (!ctx->finalized) return fail(ctx, MMPFN_ERR_STATE, "weights not finalised");
  if (!prec_ok(precision)) return fail(ctx, MMPFN_ERR_INVALID, "bad precision");
  HIPCHK(hipSetDevice(ctx->device));
  // (PREC_F16: the MGM head bank on fp16 operands, the pooler and MoE in the bf16 mode; the tokens enter the state
  // through the fp32 encoders)
  return mixer(ctx, image, S, n_mod, tokens, base_prec(precision));
}

int mmpfn_embed(mmpfn_ctx* ctx, const float* x, int S, int F, const float* tokens, int C, const float* y, int N,
                const float* uniq, int U, const float* pos_rand, int precision) {
  if (!ctx) return MMPFN_ERR_INVALID;
  HIPCHK(hipSetDevice(ctx->device));
  return embed(ctx, x, S, F, tokens, C, y, N, uniq, U, pos_rand, precision);
}

int mmpfn_run_layers(mmpfn_ctx* ctx, int l0, int l1) {
  if (!ctx) return MMPFN_ERR_INVALID;
  if (!ctx->embedded) return fail(ctx, MMPFN_ERR_STATE, "mmpfn_embed first");
  if (l0 < 0 || l1 > ctx->d.nlayers || l0 > l1) return fail(ctx, MMPFN_ERR_INVALID, "bad layer range");
  HIPCHK(hipSetDevice(ctx->device));
  for (int l = l0; l < l1; ++l) RC(run_layer(ctx, l));
  return MMPFN_OK;
}

int mmpfn_decode(mmpfn_ctx* ctx, float* logits) {
  if (!ctx || !logits) return MMPFN_ERR_INVALID;
  if (!ctx->embedded) return fail(ctx, MMPFN_ERR_STATE, "mmpfn_embed first");
  HIPCHK(hipSetDevice(ctx->device));
  return decode(ctx, logits);
}

int mmpfn_forward(mmpfn_ctx* ctx, const float* x, int S, int F, const float* tokens, int C, const float* y, int N,
                  const float* uniq, int U, const float* pos_rand, float* logits, int precision) {
  if (!ctx || !logits) return MMPFN_ERR_INVALID;
  HIPCHK(hipSetDevice(ctx->device));
  RC(embed(ctx, x, S, F, tokens, C, y, N, uniq, U, pos_rand, precision));
  for (int l = 0; l < ctx->d.nlayers; ++l) RC(run_layer(ctx, l));
  return decode(ctx, logits);
}

int mmpfn_forward_batch(mmpfn_ctx* ctx, int M, const float* const* x, int S, int F, const float* tokens, int C,
                        const float* const* y, int N, const float* const* uniq, const int* U, const float* pos_rand,
                        float* logits, int precision) {
  if (!ctx || !logits || M <= 0 || !y || !uniq || !U) return MMPFN_ERR_INVALID;
  if (F > 0 && !x) return MMPFN_ERR_INVALID;
  HIPCHK(hipSetDevice(ctx->device));
  for (int m = 0; m < M; ++m)
    RC(embed(ctx, F > 0 ? x[m] : nullptr, S, F, tokens, C, y[m], N, uniq[m], U[m], pos_rand, precision, m, M));
  for (int l = 0; l < ctx->d.nlayers; ++l) RC(run_layer(ctx, l));
  return decode(ctx, logits, M);
}

int mmpfn_state_tokens(const mmpfn_ctx* ctx) { return ctx ? ctx->T : 0; }

int mmpfn_copy_state(mmpfn_ctx* ctx, float* out, int64_t cap) {
  if (!ctx || !out) return MMPFN_ERR_INVALID;
  const int S = ctx->S, T = ctx->T, E = ctx->d.emsize;
  if (cap < (int64_t)S * T * E) return fail(ctx, MMPFN_ERR_INVALID, "state buffer too small");
  if (ctx->prec == PREC_F16) {
    HIPCHK(launch_state_f16_to_f32(ctx->ws_X.p, out, S, T, E, ctx->stream));
    return MMPFN_OK;
  }
  // [T][S][E] -> [S][T][E]
  for (int t = 0; t < T; ++t)
    HIPCHK(hipMemcpy2DAsync(out + (size_t)t * E, (size_t)T * E * 4, (const float*)ctx->ws_X.p + (size_t)t * S * E,
                            (size_t)E * 4, (size_t)E * 4, S, hipMemcpyDeviceToDevice, ctx->stream));
  return MMPFN_OK;
}

int mmpfn_aggregate(mmpfn_ctx* ctx, const float* logits, int M, int Q, int n_out, const int* perms, int n_cls,
                    float temperature, int avg_before, const float* cw, float* probs) {
  if (!ctx || !logits || !probs || M <= 0 || Q < 0 || n_out <= 0 || n_cls <= 0 || n_cls > n_out)
    return MMPFN_ERR_INVALID;
  HIPCHK(hipSetDevice(ctx->device));
  HIPCHK(launch_aggregate(logits, M, Q, n_out, perms, n_cls, temperature, avg_before, cw, probs, ctx->stream));
  return MMPFN_OK;
}

int mmpfn_status(mmpfn_ctx* ctx) {
  if (!ctx) return MMPFN_ERR_INVALID;
  HIPCHK(hipSetDevice(ctx->device));
  // wait for every stream a forward may have been queued on (lanes), not only the bound one
  for (hipStream_t s : ctx->seen_streams) HIPCHK(hipStreamSynchronize(s));
  ctx->seen_streams.assign(1, ctx->stream);
  std::vector<void*> flags{ctx->ws_flag.p};
  for (size_t i = 0; i < ctx->lanes.size(); ++i)
    if ((int)i != ctx->cur) flags.push_back(ctx->lanes[i].ws_flag.p);
  int bad = 0;
  for (void* fp : flags) {
    if (!fp) continue;
    int f = 0;
    HIPCHK(hipMemcpy(&f, fp, 4, hipMemcpyDeviceToHost));
    if (f) {
      bad |= f;
      HIPCHK(hipMemset(fp, 0, 4));  // reported once; the next forwards start clean
    }
  }
  if (bad) return fail(ctx, MMPFN_ERR_NAN, "There should be no NaNs in the encoded x and y (flag " + std::to_string(bad) + ")");
  return MMPFN_OK;
}

int mmpfn_item_attention(mmpfn_ctx* ctx, const void* q, const void* k, const void* vt, void* out, int S, int T, int H,
                         int Npad, int s0, int nq, int nk, int kvh, int precision) {
  if (!ctx || !q || !k || !vt || !out) return MMPFN_ERR_INVALID;
  if (s0 < 0 || nq < 0 || s0 + nq > S || nk <= 0 || nk > Npad || Npad % 64 || H <= 0 || T <= 0 || kvh >= H)
    return fail(ctx, MMPFN_ERR_INVALID, "bad attention geometry");
  HIPCHK(hipSetDevice(ctx->device));
  // this entry point runs the bf16 and the two fp32 element forms only (launch_attn_item); fp16 Q / K and the
  // fp8 P.V variants go through mmpfn_item_attention_layer_ex
  if (precision != PREC_F32 && precision != PREC_BF16 && precision != PREC_F32_MFMA)
    return fail(ctx, MMPFN_ERR_INVALID, "bad precision (PREC_F32, PREC_BF16 or PREC_F32_MFMA; 16-bit / fp8 Q.K forms: "
                                        "mmpfn_item_attention_layer_ex)");
  HIPCHK(launch_attn_item(q, k, vt, out, S, T, H, Npad, s0, nq, nk, kvh, precision, ctx->stream));
  return MMPFN_OK;
}

int mmpfn_cache_build(mmpfn_ctx* ctx, const float* x, int N, int F, const float* tokens, int C, const float* y_train,
                      const float* uniq, int U, const float* pos_rand, int precision, mmpfn_cache** out) {
  if (!ctx || !out || !y_train || !uniq || !pos_rand) return MMPFN_ERR_INVALID;
  *out = nullptr;
  HIPCHK(hipSetDevice(ctx->device));
  if (!prec_ok(precision)) return fail(ctx, MMPFN_ERR_INVALID, "bad precision");
  precision = base_prec(precision);  // the cache keeps bf16 K / V^T: fp8 P.V codes build a bf16 cache
  RC(embed(ctx, x, N, F, tokens, C, y_train, N, uniq, U, pos_rand, precision));
  const mmpfn_model_desc& d = ctx->d;
  const int E = d.emsize, fpg = d.features_per_group, eb = prec16(ctx->prec) ? 2 : 4;
  mmpfn_cache* cc = new mmpfn_cache;
  cc->N = N, cc->F = F, cc->G = ctx->G, cc->C = C, cc->T = ctx->T, cc->Npad = ctx->Npad, cc->prec = ctx->prec;
  cc->U = U;
  hipStream_t st = ctx->stream;
  auto build = [&]() -> int {
    RC(ensure(ctx, cc->kv, (size_t)d.nlayers * 2 * cc->T * cc->Npad * 32 * eb));
    RC(ensure(ctx, cc->slots, (size_t)(cc->G + 1) * fpg * sizeof(SlotParams)));
    RC(ensure(ctx, cc->ymean, 4));
    RC(ensure(ctx, cc->uniq, (size_t)U * 4));
    RC(ensure(ctx, cc->pe, (size_t)(cc->G + C + 1) * E * 4));
    if (cc->G)
      HIPCHK(hipMemcpyAsync(cc->slots.p, ctx->ws_slots.p, (size_t)cc->G * fpg * sizeof(SlotParams),
                            hipMemcpyDeviceToDevice, st));
    HIPCHK(hipMemcpyAsync(cc->ymean.p, ctx->ws_scr.p, 4, hipMemcpyDeviceToDevice, st));
    HIPCHK(hipMemcpyAsync(cc->uniq.p, uniq, (size_t)U * 4, hipMemcpyDeviceToDevice, st));
    HIPCHK(hipMemcpyAsync(cc->pe.p, ctx->ws_pe.p, (size_t)(cc->G + C) * E * 4, hipMemcpyDeviceToDevice, st));
    ctx->cache_out = cc;
    for (int l = 0; l < d.nlayers; ++l) {
      const int rc = run_layer(ctx, l);
      if (rc) {
        ctx->cache_out = nullptr;
        return rc;
      }
    }
    ctx->cache_out = nullptr;
    return MMPFN_OK;
  };
  const int rc = build();
  if (rc) {
    (void)hipStreamSynchronize(st);
    cache_release(cc);
    return rc;
  }
  *out = cc;
  return MMPFN_OK;
}

int mmpfn_cache_predict(mmpfn_ctx* ctx, const mmpfn_cache* cache, const float* x, int Q, int F, const float* tokens,
                        int C, float* logits) {
  if (!ctx || !cache || !logits) return MMPFN_ERR_INVALID;
  HIPCHK(hipSetDevice(ctx->device));
  RC(embed_cached(ctx, cache, x, Q, F, tokens, C, cache->prec));
  ctx->cache_in = cache;
  for (int l = 0; l < ctx->d.nlayers; ++l) {
    const int rc = run_layer(ctx, l);
    if (rc) {
      ctx->cache_in = nullptr;
      return rc;
    }
  }
  ctx->cache_in = nullptr;
  return decode(ctx, logits);
}

int64_t mmpfn_cache_bytes(const mmpfn_cache* cache) {
  if (!cache) return 0;
  return (int64_t)(cache->kv.bytes + cache->slots.bytes + cache->ymean.bytes + cache->uniq.bytes + cache->pe.bytes);
}

void mmpfn_cache_free(mmpfn_ctx* ctx, mmpfn_cache* cache) {
  if (!cache) return;
  if (ctx) {
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
  }
  cache_release(cache);
}

int mmpfn_set_parity_attention_min_keys(int n, int form) { return mmpfn::set_x3_cheap_min_keys(n, form); }

int mmpfn_kernel_timing(mmpfn_ctx* ctx, int enable) {
  if (!ctx) return MMPFN_ERR_INVALID;
  if (enable) ctx->kt_used = 0, ctx->kt_flops = 0.0;
  ctx->kt_on = enable != 0;
  return MMPFN_OK;
}

int mmpfn_kernel_timing_read(mmpfn_ctx* ctx, double* total_ms, int64_t* launches, double* flops) {
  if (!ctx || !total_ms || !launches || !flops) return MMPFN_ERR_INVALID;
  HIPCHK(hipSetDevice(ctx->device));
  double tot = 0.0;
  for (size_t i = 0; i + 1 < ctx->kt_used; i += 2) {
    HIPCHK(hipEventSynchronize(ctx->kt_pool[i + 1]));
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, ctx->kt_pool[i], ctx->kt_pool[i + 1]));
    tot += ms;
  }
  *total_ms = tot, *launches = (int64_t)(ctx->kt_used / 2), *flops = ctx->kt_flops;
  return MMPFN_OK;
}

int mmpfn_item_attention_layer(mmpfn_ctx* ctx, const void* q, const void* k, const void* vt, void* out, int S, int T,
                               int H, int Npad, int N) {
  if (!ctx || !q || !k || !vt || !out) return MMPFN_ERR_INVALID;
  if (N <= 0 || N > S || N > Npad || Npad % 64 || H <= 0 || H > 8 || T <= 0)
    return fail(ctx, MMPFN_ERR_INVALID, "bad attention geometry");
  HIPCHK(hipSetDevice(ctx->device));
  HIPCHK(launch_attn_layer(q, k, vt, out, S, T, H, Npad, N, 0, N, N, S - N, 0, ctx->stream));
  return MMPFN_OK;
}

int mmpfn_item_attention_layer_ex(mmpfn_ctx* ctx, const void* q, const void* k, const void* vt, void* out, int S,
                                  int T, int H, int Npad, int N, int precision) {
  if (!ctx || !q || !k || !vt || !out) return MMPFN_ERR_INVALID;
  if (N <= 0 || N > S || N > Npad || Npad % 64 || H <= 0 || H > 8 || T <= 0)
    return fail(ctx, MMPFN_ERR_INVALID, "bad attention geometry");
  const bool qkb = (precision & MMPFN_ATTN_QK_BF16) != 0;  // the fp16 forward's form: bf16 q / k, fp16 out
  precision &= ~MMPFN_ATTN_QK_BF16;
  if (!prec_ok(precision) || !prec16(base_prec(precision)) || (qkb && base_prec(precision) != PREC_F16))
    return fail(ctx, MMPFN_ERR_INVALID, "bad precision");
  HIPCHK(hipSetDevice(ctx->device));
  const int f8 = f8_of(precision);
  if (f8) {
    const int64_t n = (int64_t)T * H * 32 * Npad;
    RC(ensure(ctx, ctx->tap_v8, (size_t)n));
    HIPCHK(launch_vt_fp8(vt, ctx->tap_v8.p, n, ctx->stream));
  }
  const bool h16 = base_prec(precision) == PREC_F16;
  HIPCHK(launch_attn_layer(q, k, vt, out, S, T, H, Npad, N, 0, N, N, S - N, 0, ctx->stream, 0, false,
                           f8 ? ctx->tap_v8.p : nullptr, f8, h16 && !qkb, h16));
  return MMPFN_OK;
}

int mmpfn_item_attention_cached(mmpfn_ctx* ctx, const void* q, const void* k0, const void* vt0, void* out, int S,
                                int T, int H, int Npad, int N) {
  if (!ctx || !q || !k0 || !vt0 || !out) return MMPFN_ERR_INVALID;
  if (S <= 0 || N <= 0 || N > Npad || Npad % 64 || H <= 0 || H > 8 || T <= 0)
    return fail(ctx, MMPFN_ERR_INVALID, "bad attention geometry");
  HIPCHK(hipSetDevice(ctx->device));
  HIPCHK(launch_attn_layer(q, k0, vt0, out, S, T, H, Npad, N, 0, 0, 0, S, 0, ctx->stream, (int64_t)Npad * 32));
  return MMPFN_OK;
}

// ---- per-sublayer taps ------------------------------------------------------------
static int tap_check(mmpfn_ctx* ctx, int layer, const void* X, int precision) {
  if (!ctx || !X) return MMPFN_ERR_INVALID;
  if (!ctx->finalized) return fail(ctx, MMPFN_ERR_STATE, "weights not finalised");
  if (layer < 0 || layer >= ctx->d.nlayers) return fail(ctx, MMPFN_ERR_INVALID, "bad layer index");
  if (!prec_ok(precision)) return fail(ctx, MMPFN_ERR_INVALID, "bad precision");
  HIPCHK(hipSetDevice(ctx->device));
  return MMPFN_OK;
}

int mmpfn_feature_attention(mmpfn_ctx* ctx, int layer, float* X, int S, int T, int precision) {
  RC(tap_check(ctx, layer, X, precision));
  if (S <= 0 || T <= 0) return fail(ctx, MMPFN_ERR_INVALID, "bad state geometry");
  RC(tap_workspace(ctx, S, T, 64));
  return state_tap(ctx, X, (int64_t)S * T * ctx->d.emsize, precision, T, [&](void* Xs, int bp) {
    return feat_sublayer(ctx, ctx->layers[layer], Xs, S, T, 1, bp);
  });
}

int mmpfn_item_attention_block(mmpfn_ctx* ctx, int layer, float* X, int S, int T, int N, int precision) {
  RC(tap_check(ctx, layer, X, precision));
  if (S <= 0 || T <= 0 || N <= 0 || N > S) return fail(ctx, MMPFN_ERR_INVALID, "bad state geometry");
  const int Npad = (N + 63) / 64 * 64;
  RC(tap_workspace(ctx, S, T, Npad));
  return state_tap(ctx, X, (int64_t)S * T * ctx->d.emsize, precision, T, [&](void* Xs, int bp) {
    return item_sublayer(ctx, layer, Xs, S, T, N, Npad, 1, bp, false, f8_of(precision));
  });
}

int mmpfn_mlp_ln(mmpfn_ctx* ctx, int layer, float* X, int64_t rows, int precision) {
  RC(tap_check(ctx, layer, X, precision));
  if (rows <= 0) return fail(ctx, MMPFN_ERR_INVALID, "bad row count");
  return state_tap(ctx, X, rows * ctx->d.emsize, precision, -1, [&](void* Xs, int bp) {
    return mlp_sublayer(ctx, ctx->layers[layer], Xs, rows, bp, nullptr);
  });
}

int mmpfn_mgm(mmpfn_ctx* ctx, const float* image, int S, int n_mod, float* tokens, int precision) {
  if (!ctx || !image || !tokens || S <= 0 || n_mod <= 0) return MMPFN_ERR_INVALID;
  if (!ctx->finalized) return fail(ctx, MMPFN_ERR_STATE, "weights not finalised");
  if (ctx->d.mixer_type != MMPFN_MIXER_MGM && ctx->d.mixer_type != MMPFN_MIXER_MGM_CAP)
    return fail(ctx, MMPFN_ERR_INVALID, "model has no MGM head bank");
  if (!prec_ok(precision)) return fail(ctx, MMPFN_ERR_INVALID, "bad precision");
  HIPCHK(hipSetDevice(ctx->device));
  const int bp = base_prec(precision);
  return mixer_mgm(ctx, image, S, n_mod, tokens, bp);
}

int mmpfn_cap(mmpfn_ctx* ctx, const float* mgm_tokens, int S, int M, float* tokens, int precision) {
  if (!ctx || !mgm_tokens || !tokens || S <= 0 || M <= 0) return MMPFN_ERR_INVALID;
  if (!ctx->finalized) return fail(ctx, MMPFN_ERR_STATE, "weights not finalised");
  if (ctx->d.mixer_type != MMPFN_MIXER_MGM_CAP) return fail(ctx, MMPFN_ERR_INVALID, "model has no CAP");
  if (!prec_ok(precision)) return fail(ctx, MMPFN_ERR_INVALID, "bad precision");
  HIPCHK(hipSetDevice(ctx->device));
  const int bp = base_prec(precision);
  return mixer_cap(ctx, mgm_tokens, S, M, tokens, bp);
}

}  // extern "C"
