// C ABI of the modality encoders (include/mmpfn_modality.h): weight packing from the reference's
// state-dict names and the native orchestration of the two towers' forwards.
//
// ViT (DinoVisionTransformer.forward_features, vision_transformer.py:214-271; blocks
// layers/block.py:93-130 with layers/attention.py:58-77, layers/mlp.py, layers/layer_scale.py):
//   im2col + GEMM (patch_embed)  -> [cls | patches] + interpolated pos_embed
//   -> depth x [X += ls1 * proj(attn(qkv(LN1 X)));  X += ls2 * fc2(GELU(fc1(LN2 X)))]
//   -> norm; x_norm_clstoken = row 0.
// Text (transformers ElectraModel: ElectraEmbeddings, then BERT-style post-LN layers):
//   LN(word + type + pos) [-> embeddings_project]
//   -> depth x [X = LN1(X + dense(attn(qkv X)));  X = LN2(X + out(GELU(inter X)))]
//   -> last_hidden_state; cls = row 0.
// Only the CLS row of the last block reaches x_norm_clstoken / last_hidden_state[:, 0]: unless
// every token's output is requested, the last block runs its attention for the CLS query alone
// and its out-projection, MLP and norms on the B CLS rows (row-wise ops: the same values).
// State: X [B * L][dim] fp32 (residual stream), GEMM operands in the compute dtype.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <map>
#include <string>
#include <utility>
#include <vector>

#include "../../include/mmpfn_modality.h"
#include "modality.h"

using namespace mmpfn;

namespace {

struct Buf {
  void* p = nullptr;
  size_t bytes = 0;
};

uint16_t to_bf16_bits(float f) {  // round-to-nearest-even, NaN preserving
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7fffffff) > 0x7f800000) return (uint16_t)((u >> 16) | 0x40);
  u += 0x7fff + ((u >> 16) & 1);
  return (uint16_t)(u >> 16);
}

struct EncLayer {
  // ViT: ln1 = norm1, ln2 = norm2 (pre-LN); text: ln1 = attention.output.LayerNorm, ln2 = output.LayerNorm
  Buf ln1g, ln1b, ln2g, ln2b, ls1, ls2;
  Buf qkv, qkv_h, qkv_b, proj, proj_h, proj_b, fc1, fc1_h, fc1_b, fc2, fc2_h, fc2_b;
};

}  // namespace

struct mmpfn_enc {
  int device = 0;
  hipStream_t stream = nullptr;
  std::string err;
  bool have_model = false, finalized = false;
  mmpfn_enc_desc d{};
  std::map<std::string, std::vector<float>> host;
  std::vector<Buf*> owned;
  std::vector<EncLayer> layers;
  int Kpad = 0;  // ViT patch GEMM K (C * P * P rounded up to 64)
  Buf pe_w, pe_wh, pe_b, cls_tok, pos, norm_g, norm_b;
  std::map<std::pair<int, int>, Buf> pos_cache;  // interpolated pos_embed per (grid h, grid w)
  Buf wemb, pemb, temb, emb_g, emb_b, eproj, eproj_h, eproj_b;
  // workspace
  Buf X, A, QKV, O, Hh, Y, Xc, Ac, Oc, Hc, Yc, kb, flag, P0;
};

namespace {

int fail(mmpfn_enc* e, int code, const std::string& msg) {
  if (e) e->err = msg;
  return code;
}

#define HIPCHK(expr)                                                                                 \
  do {                                                                                               \
    hipError_t e_ = (expr);                                                                          \
    if (e_ != hipSuccess) return fail(enc, MMPFN_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)
#define RC(expr)                      \
  do {                                \
    int rc_ = (expr);                 \
    if (rc_ != MMPFN_OK) return rc_;  \
  } while (0)

int ensure(mmpfn_enc* enc, Buf& b, size_t bytes) {
  if (b.bytes >= bytes && b.p) return MMPFN_OK;
  if (b.p) HIPCHK(hipFree(b.p));
  b.p = nullptr, b.bytes = 0;
  bytes = (bytes + 255) & ~size_t(255);
  HIPCHK(hipMalloc(&b.p, bytes));
  b.bytes = bytes;
  return MMPFN_OK;
}

int upload(mmpfn_enc* enc, Buf& b, const std::vector<float>& v, bool as_bf16) {
  if (as_bf16) {
    std::vector<uint16_t> h(v.size());
    for (size_t i = 0; i < v.size(); ++i) h[i] = to_bf16_bits(v[i]);
    RC(ensure(enc, b, h.size() * 2));
    HIPCHK(hipMemcpy(b.p, h.data(), h.size() * 2, hipMemcpyHostToDevice));
  } else {
    RC(ensure(enc, b, v.size() * 4));
    HIPCHK(hipMemcpy(b.p, v.data(), v.size() * 4, hipMemcpyHostToDevice));
  }
  return MMPFN_OK;
}

const std::vector<float>* getw(mmpfn_enc* enc, const std::string& name, size_t numel) {
  auto it = enc->host.find(name);
  if (it == enc->host.end()) {
    enc->err = "missing weight: " + name;
    return nullptr;
  }
  if (it->second.size() != numel) {
    enc->err = "weight " + name + " has " + std::to_string(it->second.size()) + " elements, expected " +
               std::to_string(numel);
    return nullptr;
  }
  return &it->second;
}

#define GETW(var, name, n)                                  \
  const std::vector<float>* var = getw(enc, (name), (n));   \
  if (!var) return MMPFN_ERR_WEIGHT;

// a Linear's weight in both dtypes (fp32 for the parity mode, bf16 for the MFMA path) + bias
int up_linear(mmpfn_enc* enc, Buf& w, Buf& wh, Buf& b, const std::vector<float>& wv, const std::vector<float>& bv) {
  RC(upload(enc, w, wv, false));
  RC(upload(enc, wh, wv, true));
  RC(upload(enc, b, bv, false));
  return MMPFN_OK;
}

int finalize_vit(mmpfn_enc* enc) {
  const auto& d = enc->d;
  const int D = d.dim, F = d.mlp_hidden, P = d.patch, C = d.in_chans, M = d.pos_grid;
  const int K0 = C * P * P;
  enc->Kpad = (K0 + 63) / 64 * 64;
  {
    GETW(w, "patch_embed.proj.weight", (size_t)D * K0);
    GETW(b, "patch_embed.proj.bias", (size_t)D);
    std::vector<float> wp((size_t)D * enc->Kpad, 0.f);
    for (int n = 0; n < D; ++n)
      for (int k = 0; k < K0; ++k) wp[(size_t)n * enc->Kpad + k] = (*w)[(size_t)n * K0 + k];
    RC(up_linear(enc, enc->pe_w, enc->pe_wh, enc->pe_b, wp, *b));
  }
  {
    GETW(c, "cls_token", (size_t)D);
    GETW(p, "pos_embed", (size_t)(1 + M * M) * D);
    GETW(g, "norm.weight", (size_t)D);
    GETW(b, "norm.bias", (size_t)D);
    RC(upload(enc, enc->cls_tok, *c, false));
    RC(upload(enc, enc->pos, *p, false));
    RC(upload(enc, enc->norm_g, *g, false));
    RC(upload(enc, enc->norm_b, *b, false));
  }
  enc->layers.assign(d.depth, EncLayer{});
  for (int i = 0; i < d.depth; ++i) {
    const std::string pre = "blocks." + std::to_string(i) + ".";
    EncLayer& L = enc->layers[i];
    GETW(n1g, pre + "norm1.weight", D);
    GETW(n1b, pre + "norm1.bias", D);
    GETW(n2g, pre + "norm2.weight", D);
    GETW(n2b, pre + "norm2.bias", D);
    GETW(qw, pre + "attn.qkv.weight", (size_t)3 * D * D);
    GETW(qb, pre + "attn.qkv.bias", (size_t)3 * D);
    GETW(pw, pre + "attn.proj.weight", (size_t)D * D);
    GETW(pb, pre + "attn.proj.bias", D);
    GETW(f1w, pre + "mlp.fc1.weight", (size_t)F * D);
    GETW(f1b, pre + "mlp.fc1.bias", F);
    GETW(f2w, pre + "mlp.fc2.weight", (size_t)D * F);
    GETW(f2b, pre + "mlp.fc2.bias", D);
    RC(upload(enc, L.ln1g, *n1g, false));
    RC(upload(enc, L.ln1b, *n1b, false));
    RC(upload(enc, L.ln2g, *n2g, false));
    RC(upload(enc, L.ln2b, *n2b, false));
    RC(up_linear(enc, L.qkv, L.qkv_h, L.qkv_b, *qw, *qb));
    RC(up_linear(enc, L.proj, L.proj_h, L.proj_b, *pw, *pb));
    RC(up_linear(enc, L.fc1, L.fc1_h, L.fc1_b, *f1w, *f1b));
    RC(up_linear(enc, L.fc2, L.fc2_h, L.fc2_b, *f2w, *f2b));
    if (d.layerscale) {
      GETW(g1, pre + "ls1.gamma", D);
      GETW(g2, pre + "ls2.gamma", D);
      RC(upload(enc, L.ls1, *g1, false));
      RC(upload(enc, L.ls2, *g2, false));
    }
  }
  return MMPFN_OK;
}

int finalize_text(mmpfn_enc* enc) {
  const auto& d = enc->d;
  const int D = d.dim, F = d.mlp_hidden, E = d.embedding_size;
  {
    GETW(w, "embeddings.word_embeddings.weight", (size_t)d.vocab * E);
    GETW(p, "embeddings.position_embeddings.weight", (size_t)d.max_pos * E);
    GETW(t, "embeddings.token_type_embeddings.weight", (size_t)d.type_vocab * E);
    GETW(g, "embeddings.LayerNorm.weight", E);
    GETW(b, "embeddings.LayerNorm.bias", E);
    RC(upload(enc, enc->wemb, *w, false));
    RC(upload(enc, enc->pemb, *p, false));
    RC(upload(enc, enc->temb, *t, false));
    RC(upload(enc, enc->emb_g, *g, false));
    RC(upload(enc, enc->emb_b, *b, false));
    if (E != D) {
      GETW(pw, "embeddings_project.weight", (size_t)D * E);
      GETW(pb, "embeddings_project.bias", D);
      RC(up_linear(enc, enc->eproj, enc->eproj_h, enc->eproj_b, *pw, *pb));
    }
  }
  enc->layers.assign(d.depth, EncLayer{});
  for (int i = 0; i < d.depth; ++i) {
    const std::string pre = "encoder.layer." + std::to_string(i) + ".";
    EncLayer& L = enc->layers[i];
    GETW(qw, pre + "attention.self.query.weight", (size_t)D * D);
    GETW(qb, pre + "attention.self.query.bias", D);
    GETW(kw, pre + "attention.self.key.weight", (size_t)D * D);
    GETW(kb, pre + "attention.self.key.bias", D);
    GETW(vw, pre + "attention.self.value.weight", (size_t)D * D);
    GETW(vb, pre + "attention.self.value.bias", D);
    GETW(ow, pre + "attention.output.dense.weight", (size_t)D * D);
    GETW(ob, pre + "attention.output.dense.bias", D);
    GETW(l1g, pre + "attention.output.LayerNorm.weight", D);
    GETW(l1b, pre + "attention.output.LayerNorm.bias", D);
    GETW(iw, pre + "intermediate.dense.weight", (size_t)F * D);
    GETW(ib, pre + "intermediate.dense.bias", F);
    GETW(o2w, pre + "output.dense.weight", (size_t)D * F);
    GETW(o2b, pre + "output.dense.bias", D);
    GETW(l2g, pre + "output.LayerNorm.weight", D);
    GETW(l2b, pre + "output.LayerNorm.bias", D);
    std::vector<float> w3(*qw), b3(*qb);  // [q | k | v] rows: one QKV GEMM
    w3.insert(w3.end(), kw->begin(), kw->end());
    w3.insert(w3.end(), vw->begin(), vw->end());
    b3.insert(b3.end(), kb->begin(), kb->end());
    b3.insert(b3.end(), vb->begin(), vb->end());
    RC(up_linear(enc, L.qkv, L.qkv_h, L.qkv_b, w3, b3));
    RC(up_linear(enc, L.proj, L.proj_h, L.proj_b, *ow, *ob));
    RC(up_linear(enc, L.fc1, L.fc1_h, L.fc1_b, *iw, *ib));
    RC(up_linear(enc, L.fc2, L.fc2_h, L.fc2_b, *o2w, *o2b));
    RC(upload(enc, L.ln1g, *l1g, false));
    RC(upload(enc, L.ln1b, *l1b, false));
    RC(upload(enc, L.ln2g, *l2g, false));
    RC(upload(enc, L.ln2b, *l2b, false));
  }
  return MMPFN_OK;
}

inline const void* Wsel(const Buf& f, const Buf& h, int prec) { return prec == PREC_BF16 ? h.p : f.p; }

// C = A . W^T + bias, epilogue per mode; fp32 parity mode: the generic fp32-MFMA GEMM (gemm.hip)
// into Y, then the residual / store step
int linear(mmpfn_enc* enc, int prec, const void* A, const Buf& Wf, const Buf& Wh, const Buf& bias, int M, int N,
           int K, int epi, int act, void* C, const float* gamma, float* Y) {
  if (M <= 0) return MMPFN_OK;
  if (prec == PREC_BF16) {
    HIPCHK(launch_gemm_tile(A, Wh.p, (const float*)bias.p, gamma, C, N, M, N, K, epi, act, enc->stream));
    return MMPFN_OK;
  }
  if (N % 192 != 0) return fail(enc, MMPFN_ERR_INVALID, "fp32 mode needs linear widths that are multiples of 192");
  GemmArgs g;
  std::memset(&g, 0, sizeof(g));
  g.a_rdiv = 1ll << 62, g.a_rmul = 0, g.a_rmul2 = 1, g.rdiv2 = 1ll << 62, g.ln_eps = 1e-5f;
  g.A = A, g.lda = K, g.W = Wf.p, g.bias = (const float*)bias.p, g.M = M, g.N = N, g.K = K, g.act = act;
  g.C = epi == GT_RESID ? (void*)Y : C, g.ldc = N;
  // the encoders' fp32 mode stays on fp32-input MFMA (their 1-2e-6 parity; the tower runs once per dataset)
  HIPCHK(launch_gemm(g, PREC_F32_MFMA, EPI_STORE, true, true, 1, enc->stream));
  if (epi == GT_RESID) HIPCHK(launch_resid((float*)C, Y, gamma, M, N, enc->stream));
  return MMPFN_OK;
}

// workspace for B sequences of L tokens (rows M = B * L)
int ensure_ws(mmpfn_enc* enc, int64_t M, int B, int prec) {
  const int64_t D = enc->d.dim, F = enc->d.mlp_hidden;
  const int eb = prec == PREC_BF16 ? 2 : 4;
  RC(ensure(enc, enc->X, M * D * 4));
  RC(ensure(enc, enc->A, M * std::max<int64_t>(D, enc->Kpad) * eb));
  RC(ensure(enc, enc->QKV, M * 3 * D * eb));
  RC(ensure(enc, enc->O, M * D * eb));
  RC(ensure(enc, enc->Hh, M * F * eb));
  RC(ensure(enc, enc->Y, (prec == PREC_BF16 ? 1 : M) * D * 4));
  RC(ensure(enc, enc->Xc, (int64_t)B * D * 4));
  RC(ensure(enc, enc->Ac, (int64_t)B * D * eb));
  RC(ensure(enc, enc->Oc, (int64_t)B * D * eb));
  RC(ensure(enc, enc->Hc, (int64_t)B * F * eb));
  RC(ensure(enc, enc->Yc, (int64_t)B * D * 4));
  return MMPFN_OK;
}

// the interpolated positional table for a (gh, gw) patch grid (interpolate_pos_encoding,
// vision_transformer.py:180-212), computed on the device once per grid
int pos_for(mmpfn_enc* enc, int gh, int gw, const float** out) {
  const auto& d = enc->d;
  const int M = d.pos_grid, D = d.dim;
  if (gh == M && gw == M) {
    *out = (const float*)enc->pos.p;
    return MMPFN_OK;
  }
  auto key = std::make_pair(gh, gw);
  auto it = enc->pos_cache.find(key);
  if (it == enc->pos_cache.end()) {
    Buf b;
    RC(ensure(enc, b, (size_t)(1 + gh * gw) * D * 4));
    // torch upsample_bicubic2d source scale: 1 / scale_factor (double -> float) when the reference
    // passes scale factors ((g + offset) / M), else input / output
    float sh, sw;
    if (d.interp_offset != 0.0) {
      sh = (float)(1.0 / (((double)gh + d.interp_offset) / M));
      sw = (float)(1.0 / (((double)gw + d.interp_offset) / M));
    } else {
      sh = (float)M / (float)gh;
      sw = (float)M / (float)gw;
    }
    HIPCHK(launch_pos_interp((const float*)enc->pos.p, M, D, gh, gw, sh, sw, (float*)b.p, enc->stream));
    it = enc->pos_cache.emplace(key, b).first;
  }
  *out = (const float*)it->second.p;
  return MMPFN_OK;
}

// the last block on the B CLS rows: Xc <- row 0 of every sequence, then the block's out-projection,
// MLP and norms on those rows (pre-LN ViT or post-LN text)
int cls_tail(mmpfn_enc* enc, const EncLayer& Lw, int B, int64_t L, int prec, bool post_ln) {
  const int D = enc->d.dim, F = enc->d.mlp_hidden;
  const float eps = enc->d.ln_eps;
  hipStream_t st = enc->stream;
  HIPCHK(launch_gather_rows(enc->X.p, L * D, B, D, enc->Xc.p, 4, st));
  float* Xc = (float*)enc->Xc.p;
  RC(linear(enc, prec, enc->Oc.p, Lw.proj, Lw.proj_h, Lw.proj_b, B, D, D, GT_RESID, 0, Xc,
            post_ln ? nullptr : (const float*)Lw.ls1.p, (float*)enc->Yc.p));
  const bool bf = prec == PREC_BF16;
  if (post_ln) {
    HIPCHK(launch_ln_dual(Xc, B, D, eps, Xc, bf ? enc->Ac.p : nullptr, (const float*)Lw.ln1g.p,
                          (const float*)Lw.ln1b.p, st));
  } else {
    HIPCHK(launch_ln_dual(Xc, B, D, eps, bf ? nullptr : (float*)enc->Ac.p, bf ? enc->Ac.p : nullptr,
                          (const float*)Lw.ln2g.p, (const float*)Lw.ln2b.p, st));
  }
  const void* Ain = post_ln && !bf ? (const void*)Xc : enc->Ac.p;
  RC(linear(enc, prec, Ain, Lw.fc1, Lw.fc1_h, Lw.fc1_b, B, F, D, GT_BF16, 1, enc->Hc.p, nullptr, nullptr));
  RC(linear(enc, prec, enc->Hc.p, Lw.fc2, Lw.fc2_h, Lw.fc2_b, B, D, F, GT_RESID, 0, Xc,
            post_ln ? nullptr : (const float*)Lw.ls2.p, (float*)enc->Yc.p));
  if (post_ln)
    HIPCHK(launch_ln_dual(Xc, B, D, eps, Xc, nullptr, (const float*)Lw.ln2g.p, (const float*)Lw.ln2b.p, st));
  return MMPFN_OK;
}

int check_desc(mmpfn_enc* enc, const mmpfn_enc_desc& d) {
  if (d.kind != MMPFN_ENC_VIT && d.kind != MMPFN_ENC_TEXT) return fail(enc, MMPFN_ERR_INVALID, "unknown encoder kind");
  if (d.dim <= 0 || d.heads <= 0 || d.dim != 64 * d.heads)
    return fail(enc, MMPFN_ERR_INVALID, "head_dim must be 64 (dim = 64 * heads)");
  if (d.dim % 256 || d.mlp_hidden <= 0 || d.mlp_hidden % 256 || d.depth <= 0 || d.dim > 1024)
    return fail(enc, MMPFN_ERR_INVALID, "dim and mlp_hidden must be multiples of 256 (dim <= 1024), depth > 0");
  if (!(d.ln_eps > 0.f)) return fail(enc, MMPFN_ERR_INVALID, "ln_eps must be > 0");
  if (d.kind == MMPFN_ENC_VIT && (d.patch <= 0 || d.in_chans <= 0 || d.pos_grid <= 0))
    return fail(enc, MMPFN_ERR_INVALID, "patch, in_chans and pos_grid must be > 0");
  if (d.kind == MMPFN_ENC_TEXT &&
      (d.vocab <= 0 || d.max_pos <= 0 || d.type_vocab <= 0 || d.embedding_size <= 0 || d.embedding_size % 4 ||
       d.embedding_size > 1024 || (d.embedding_size != d.dim && d.embedding_size % 32)))
    return fail(enc, MMPFN_ERR_INVALID, "bad text-encoder sizes");
  return MMPFN_OK;
}

}  // namespace

extern "C" {

mmpfn_enc* mmpfn_enc_create(int device, void* hip_stream) {
  if (hipSetDevice(device) != hipSuccess) return nullptr;
  mmpfn_enc* e = new mmpfn_enc();
  e->device = device;
  e->stream = (hipStream_t)hip_stream;
  return e;
}

void mmpfn_enc_destroy(mmpfn_enc* enc) {
  if (!enc) return;
  (void)hipSetDevice(enc->device);
  auto freeb = [](Buf& b) {
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
  };
  for (auto& L : enc->layers)
    for (Buf* b : {&L.ln1g, &L.ln1b, &L.ln2g, &L.ln2b, &L.ls1, &L.ls2, &L.qkv, &L.qkv_h, &L.qkv_b, &L.proj,
                   &L.proj_h, &L.proj_b, &L.fc1, &L.fc1_h, &L.fc1_b, &L.fc2, &L.fc2_h, &L.fc2_b})
      freeb(*b);
  for (auto& kv : enc->pos_cache) freeb(kv.second);
  for (Buf* b : {&enc->pe_w, &enc->pe_wh, &enc->pe_b, &enc->cls_tok, &enc->pos, &enc->norm_g, &enc->norm_b,
                 &enc->wemb, &enc->pemb, &enc->temb, &enc->emb_g, &enc->emb_b, &enc->eproj, &enc->eproj_h,
                 &enc->eproj_b, &enc->X, &enc->A, &enc->QKV, &enc->O, &enc->Hh, &enc->Y, &enc->Xc, &enc->Ac,
                 &enc->Oc, &enc->Hc, &enc->Yc, &enc->kb, &enc->flag, &enc->P0})
    freeb(*b);
  delete enc;
}

const char* mmpfn_enc_last_error(const mmpfn_enc* enc) { return enc ? enc->err.c_str() : "null encoder"; }

int mmpfn_enc_set_stream(mmpfn_enc* enc, void* hip_stream) {
  if (!enc) return MMPFN_ERR_INVALID;
  enc->stream = (hipStream_t)hip_stream;
  return MMPFN_OK;
}

int mmpfn_enc_set_model(mmpfn_enc* enc, const mmpfn_enc_desc* desc) {
  if (!enc || !desc) return MMPFN_ERR_INVALID;
  RC(check_desc(enc, *desc));
  enc->d = *desc;
  enc->have_model = true;
  enc->finalized = false;
  enc->host.clear();
  return MMPFN_OK;
}

int mmpfn_enc_load_weight(mmpfn_enc* enc, const char* name, const float* host_data, int64_t numel) {
  if (!enc || !name || (numel > 0 && !host_data) || numel < 0) return MMPFN_ERR_INVALID;
  if (!enc->have_model) return fail(enc, MMPFN_ERR_STATE, "mmpfn_enc_set_model first");
  enc->host[name].assign(host_data, host_data + numel);
  enc->finalized = false;
  return MMPFN_OK;
}

int mmpfn_enc_finalize(mmpfn_enc* enc) {
  if (!enc) return MMPFN_ERR_INVALID;
  if (!enc->have_model) return fail(enc, MMPFN_ERR_STATE, "mmpfn_enc_set_model first");
  HIPCHK(hipSetDevice(enc->device));
  RC(enc->d.kind == MMPFN_ENC_VIT ? finalize_vit(enc) : finalize_text(enc));
  HIPCHK(hipDeviceSynchronize());
  enc->host.clear();
  enc->finalized = true;
  return MMPFN_OK;
}

int mmpfn_vit_forward(mmpfn_enc* enc, const float* images, int B, int H, int W, float* cls, float* tokens,
                      int precision) {
  if (!enc) return MMPFN_ERR_INVALID;
  if (!enc->finalized || enc->d.kind != MMPFN_ENC_VIT) return fail(enc, MMPFN_ERR_STATE, "no finalized ViT model");
  const auto& d = enc->d;
  const int P = d.patch, D = d.dim, F = d.mlp_hidden, nh = d.heads;
  if (B <= 0 || !images || !cls || H <= 0 || W <= 0 || H % P || W % P)
    return fail(enc, MMPFN_ERR_INVALID, "images must be [B][C][H][W] with H, W multiples of the patch size");
  if (precision != PREC_F32 && precision != PREC_BF16) return fail(enc, MMPFN_ERR_INVALID, "bad precision");
  const int prec = precision;
  const bool bf = prec == PREC_BF16;
  const int gh = H / P, gw = W / P, np = gh * gw;
  const int64_t L = 1 + np, M = (int64_t)B * L;
  if (M > 0x7fffffffll) return fail(enc, MMPFN_ERR_INVALID, "batch too large");
  const float eps = d.ln_eps;
  hipStream_t st = enc->stream;
  HIPCHK(hipSetDevice(enc->device));
  RC(ensure_ws(enc, M, B, prec));
  RC(ensure(enc, enc->P0, (size_t)B * np * D * 4));
  const float* pe = nullptr;
  RC(pos_for(enc, gh, gw, &pe));
  // patch embedding: im2col + GEMM (+ bias) -> [cls | patches] + pos
  HIPCHK(launch_im2col(images, B, d.in_chans, H, W, P, enc->Kpad, enc->A.p, !bf, st));
  RC(linear(enc, prec, enc->A.p, enc->pe_w, enc->pe_wh, enc->pe_b, B * np, D, enc->Kpad, GT_F32, 0, enc->P0.p,
            nullptr, nullptr));
  float* X = (float*)enc->X.p;
  HIPCHK(launch_vit_assemble((const float*)enc->P0.p, (const float*)enc->cls_tok.p, pe, B, np, D, X, st));
  for (int i = 0; i < d.depth; ++i) {
    const EncLayer& Lw = enc->layers[i];
    const bool tail = i == d.depth - 1 && tokens == nullptr;
    // X += ls1 * attn(norm1(X))   (block.py:106-115)
    HIPCHK(launch_ln_dual(X, M, D, eps, bf ? nullptr : (float*)enc->A.p, bf ? enc->A.p : nullptr,
                          (const float*)Lw.ln1g.p, (const float*)Lw.ln1b.p, st));
    RC(linear(enc, prec, enc->A.p, Lw.qkv, Lw.qkv_h, Lw.qkv_b, (int)M, 3 * D, D, GT_BF16, 0, enc->QKV.p, nullptr,
              nullptr));
    if (tail) {
      HIPCHK(launch_attn64(enc->QKV.p, nullptr, enc->Oc.p, B, (int)L, nh, 0, 1, 1, prec, st));
      RC(cls_tail(enc, Lw, B, L, prec, false));
      break;
    }
    HIPCHK(launch_attn64(enc->QKV.p, nullptr, enc->O.p, B, (int)L, nh, 0, (int)L, L, prec, st));
    RC(linear(enc, prec, enc->O.p, Lw.proj, Lw.proj_h, Lw.proj_b, (int)M, D, D, GT_RESID, 0, X,
              (const float*)Lw.ls1.p, (float*)enc->Y.p));
    // X += ls2 * mlp(norm2(X))
    HIPCHK(launch_ln_dual(X, M, D, eps, bf ? nullptr : (float*)enc->A.p, bf ? enc->A.p : nullptr,
                          (const float*)Lw.ln2g.p, (const float*)Lw.ln2b.p, st));
    RC(linear(enc, prec, enc->A.p, Lw.fc1, Lw.fc1_h, Lw.fc1_b, (int)M, F, D, GT_BF16, 1, enc->Hh.p, nullptr, nullptr));
    RC(linear(enc, prec, enc->Hh.p, Lw.fc2, Lw.fc2_h, Lw.fc2_b, (int)M, D, F, GT_RESID, 0, X,
              (const float*)Lw.ls2.p, (float*)enc->Y.p));
  }
  // x_norm = norm(x); x_norm_clstoken = x_norm[:, 0]
  if (tokens) {
    HIPCHK(launch_ln_dual(X, M, D, eps, tokens, nullptr, (const float*)enc->norm_g.p, (const float*)enc->norm_b.p, st));
    HIPCHK(launch_gather_rows(tokens, L * D, B, D, cls, 4, st));
  } else {
    HIPCHK(launch_ln_dual((const float*)enc->Xc.p, B, D, eps, cls, nullptr, (const float*)enc->norm_g.p,
                          (const float*)enc->norm_b.p, st));
  }
  return MMPFN_OK;
}

int mmpfn_enc_attention(mmpfn_enc* enc, const void* qkv, const float* kbias, void* out, int B, int L, int H,
                        int precision) {
  if (!enc) return MMPFN_ERR_INVALID;
  if (!qkv || !out || B <= 0 || L <= 0 || H <= 0) return fail(enc, MMPFN_ERR_INVALID, "qkv, out and B, L, H > 0");
  if (precision != PREC_F32 && precision != PREC_BF16) return fail(enc, MMPFN_ERR_INVALID, "bad precision");
  HIPCHK(hipSetDevice(enc->device));
  HIPCHK(launch_attn64(qkv, kbias, out, B, L, H, 0, L, L, precision, enc->stream));
  return MMPFN_OK;
}

int mmpfn_text_forward(mmpfn_enc* enc, const int32_t* ids, const int32_t* mask, const int32_t* types, int B, int L,
                       float* cls, float* hidden, int precision) {
  if (!enc) return MMPFN_ERR_INVALID;
  if (!enc->finalized || enc->d.kind != MMPFN_ENC_TEXT) return fail(enc, MMPFN_ERR_STATE, "no finalized text model");
  const auto& d = enc->d;
  const int D = d.dim, F = d.mlp_hidden, E = d.embedding_size, nh = d.heads;
  if (B <= 0 || L <= 0 || !ids || !cls) return fail(enc, MMPFN_ERR_INVALID, "ids [B][L] and cls are required");
  if (L > d.max_pos) return fail(enc, MMPFN_ERR_INVALID, "sequence longer than max_position_embeddings");
  if (precision != PREC_F32 && precision != PREC_BF16) return fail(enc, MMPFN_ERR_INVALID, "bad precision");
  const int prec = precision;
  const bool bf = prec == PREC_BF16;
  const int64_t M = (int64_t)B * L;
  const float eps = d.ln_eps;
  hipStream_t st = enc->stream;
  HIPCHK(hipSetDevice(enc->device));
  RC(ensure_ws(enc, M, B, prec));
  RC(ensure(enc, enc->flag, 256));
  HIPCHK(hipMemsetAsync(enc->flag.p, 0, 4, st));
  const float* kbias = nullptr;
  if (mask) {
    RC(ensure(enc, enc->kb, M * 4));
    HIPCHK(launch_mask_bias(mask, (float*)enc->kb.p, M, st));
    kbias = (const float*)enc->kb.p;
  }
  float* X = (float*)enc->X.p;
  if (E == D) {
    HIPCHK(launch_text_embed(ids, types, M, L, E, (const float*)enc->wemb.p, (const float*)enc->pemb.p,
                             (const float*)enc->temb.p, (const float*)enc->emb_g.p, (const float*)enc->emb_b.p,
                             eps, X, bf ? enc->A.p : nullptr, d.vocab, d.type_vocab, (int*)enc->flag.p, st));
  } else {  // LN(embeddings) [M][E] -> embeddings_project -> X
    RC(ensure(enc, enc->P0, (size_t)M * E * 4 + (size_t)M * E * 2));
    float* e32 = (float*)enc->P0.p;
    void* e16 = (char*)enc->P0.p + (size_t)M * E * 4;
    HIPCHK(launch_text_embed(ids, types, M, L, E, (const float*)enc->wemb.p, (const float*)enc->pemb.p,
                             (const float*)enc->temb.p, (const float*)enc->emb_g.p, (const float*)enc->emb_b.p,
                             eps, e32, bf ? e16 : nullptr, d.vocab, d.type_vocab, (int*)enc->flag.p, st));
    if (bf) {
      HIPCHK(launch_gemm_tile(e16, enc->eproj_h.p, (const float*)enc->eproj_b.p, nullptr, X, D, (int)M, D, E,
                              GT_F32, 0, st));
      HIPCHK(launch_cast_bf16(X, enc->A.p, M * D, st));
    } else {
      RC(linear(enc, prec, e32, enc->eproj, enc->eproj_h, enc->eproj_b, (int)M, D, E, GT_F32, 0, X, nullptr,
                nullptr));
    }
  }
  for (int i = 0; i < d.depth; ++i) {
    const EncLayer& Lw = enc->layers[i];
    const bool tail = i == d.depth - 1 && hidden == nullptr;
    // X = LN1(X + dense(attn(qkv(X))))   (ElectraSelfAttention / ElectraSelfOutput)
    const void* Ain = bf ? enc->A.p : (const void*)X;
    RC(linear(enc, prec, Ain, Lw.qkv, Lw.qkv_h, Lw.qkv_b, (int)M, 3 * D, D, GT_BF16, 0, enc->QKV.p, nullptr, nullptr));
    if (tail) {
      HIPCHK(launch_attn64(enc->QKV.p, kbias, enc->Oc.p, B, L, nh, 0, 1, 1, prec, st));
      RC(cls_tail(enc, Lw, B, L, prec, true));
      break;
    }
    HIPCHK(launch_attn64(enc->QKV.p, kbias, enc->O.p, B, L, nh, 0, L, L, prec, st));
    RC(linear(enc, prec, enc->O.p, Lw.proj, Lw.proj_h, Lw.proj_b, (int)M, D, D, GT_RESID, 0, X, nullptr,
              (float*)enc->Y.p));
    HIPCHK(launch_ln_dual(X, M, D, eps, X, bf ? enc->A.p : nullptr, (const float*)Lw.ln1g.p, (const float*)Lw.ln1b.p, st));
    // X = LN2(X + out(GELU(inter(X))))   (ElectraIntermediate / ElectraOutput)
    RC(linear(enc, prec, Ain, Lw.fc1, Lw.fc1_h, Lw.fc1_b, (int)M, F, D, GT_BF16, 1, enc->Hh.p, nullptr, nullptr));
    RC(linear(enc, prec, enc->Hh.p, Lw.fc2, Lw.fc2_h, Lw.fc2_b, (int)M, D, F, GT_RESID, 0, X, nullptr,
              (float*)enc->Y.p));
    HIPCHK(launch_ln_dual(X, M, D, eps, X, bf ? enc->A.p : nullptr, (const float*)Lw.ln2g.p, (const float*)Lw.ln2b.p, st));
  }
  if (hidden) {
    HIPCHK(hipMemcpyAsync(hidden, X, M * D * 4, hipMemcpyDeviceToDevice, st));
    HIPCHK(launch_gather_rows(X, (int64_t)L * D, B, D, cls, 4, st));
  } else {
    HIPCHK(hipMemcpyAsync(cls, enc->Xc.p, (size_t)B * D * 4, hipMemcpyDeviceToDevice, st));
  }
  int flag = 0;
  HIPCHK(hipMemcpyAsync(&flag, enc->flag.p, 4, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  if (flag) return fail(enc, MMPFN_ERR_INVALID, "input id or token type out of range (the reference's lookup raises)");
  return MMPFN_OK;
}

}  // extern "C"
