/*
 * mmpfn_modality.h -- C-ABI of the MI355X (gfx950) modality encoders.
 *
 * The reference computes its modality tokens `image [S, n_mod, 768]` once per dataset with two
 * pretrained towers and caches them as `.pt` files:
 *   - image: DINOv2 ViT-B/14 CLS (mmpfn/datasets/pad_ufes_20.py:66-107, petfinder.py:100-146):
 *       vit_base(patch_size=14, img_size=518, init_values=1.0, num_register_tokens=0, block_chunks=0)
 *       .forward_features(x)["x_norm_clstoken"]      (models/dino_v2/models/vision_transformer.py:255-271)
 *   - text: ELECTRA-base CLS (petfinder.py:150-181):
 *       ElectraModel(**tokenizer(text)).last_hidden_state[:, 0, :]   (transformers' ElectraModel)
 * This library runs both towers on the device: weights by the reference's state-dict names,
 * inputs and outputs as device pointers on the caller's HIP stream, one context per tower.
 *
 * Conventions as in mmpfn_hip.h: int status (0 ok, negative MMPFN_ERR_*), detail from
 * mmpfn_enc_last_error; precision MMPFN_PREC_F32 (fp32 everywhere, the reference's arithmetic) or
 * MMPFN_PREC_BF16 (bf16 MFMA operands, fp32 accumulate / residual / LayerNorm / softmax).
 * Supported geometry: head_dim 64 (dim = 64 * heads), dim % 256 == 0, mlp_hidden % 256 == 0; the fp32
 * mode also needs dim and mlp_hidden % 192 == 0 (ViT-B / ELECTRA-base: 768, 3072).
 */
#ifndef MMPFN_MODALITY_H_
#define MMPFN_MODALITY_H_

#include <stdint.h>

#include "mmpfn_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

#define MMPFN_ENC_VIT 1  /* DinoVisionTransformer: pre-LN blocks with LayerScale (layers/block.py:93-130) */
#define MMPFN_ENC_TEXT 2 /* ElectraModel: embeddings + post-LN BERT layers */

typedef struct mmpfn_enc mmpfn_enc;

typedef struct mmpfn_enc_desc {
  int kind;        /* MMPFN_ENC_* */
  int dim;         /* embed_dim / hidden_size */
  int depth;       /* blocks / num_hidden_layers */
  int heads;       /* num_heads / num_attention_heads (head_dim must be 64) */
  int mlp_hidden;  /* mlp_ratio * dim / intermediate_size */
  float ln_eps;    /* 1e-6 (DINOv2 norm_layer) / layer_norm_eps (1e-12) */
  /* ViT */
  int patch;             /* patch_size (14) */
  int in_chans;          /* 3 */
  int pos_grid;          /* M of pos_embed [1, 1 + M*M, dim] (img_size 518 / 14 = 37) */
  double interp_offset;  /* interpolate_offset (0.1, as the reference's Python float); 0 = exact size */
  int layerscale;        /* init_values set: ls1.gamma / ls2.gamma present */
  /* text */
  int vocab;             /* vocab_size */
  int max_pos;           /* max_position_embeddings */
  int type_vocab;        /* type_vocab_size */
  int embedding_size;    /* embedding_size (== dim: no embeddings_project) */
} mmpfn_enc_desc;

mmpfn_enc* mmpfn_enc_create(int device, void* hip_stream);
void mmpfn_enc_destroy(mmpfn_enc* enc);
const char* mmpfn_enc_last_error(const mmpfn_enc* enc);
int mmpfn_enc_set_stream(mmpfn_enc* enc, void* hip_stream);
int mmpfn_enc_set_model(mmpfn_enc* enc, const mmpfn_enc_desc* desc);
/* one tensor of the reference state dict, fp32 host data (e.g. "blocks.3.attn.qkv.weight",
 * "encoder.layer.0.attention.self.query.weight") */
int mmpfn_enc_load_weight(mmpfn_enc* enc, const char* name, const float* host_data, int64_t numel);
int mmpfn_enc_finalize(mmpfn_enc* enc); /* pack / convert / upload; synchronous */

/* DinoVisionTransformer.forward_features (vision_transformer.py:214-271): images [B][C][H][W] fp32
 * (H, W multiples of the patch), cls [B][dim] fp32 = x_norm_clstoken; tokens (optional, may be NULL)
 * [B][1 + H*W/P^2][dim] fp32 = x_norm of every token (cls then patches). */
int mmpfn_vit_forward(mmpfn_enc* enc, const float* images, int B, int H, int W, float* cls, float* tokens,
                      int precision);

/* ElectraModel.forward(input_ids, attention_mask, token_type_ids) (transformers modeling_electra):
 * ids / mask / types [B][L] int32 (mask, types may be NULL: all ones / zeros; mask 0 excludes the
 * key), cls [B][dim] fp32 = last_hidden_state[:, 0]; hidden (optional) [B][L][dim] fp32 =
 * last_hidden_state.  Out-of-range ids / types -> MMPFN_ERR_INVALID (the reference's lookup raises). */
int mmpfn_text_forward(mmpfn_enc* enc, const int32_t* ids, const int32_t* mask, const int32_t* types, int B, int L,
                       float* cls, float* hidden, int precision);

/* Kernel tap (tests, diagnostics): the towers' self-attention (layers/attention.py:58-77; the text tower's
 * masked BERT attention) on device buffers: qkv [B][L][3][H][64] (the QKV GEMM's rows: q | k | v), kbias
 * [B][L] fp32 additive key bias in natural-log units (-inf excludes the key) or NULL, out [B][L][H*64];
 * bf16 qkv / out for MMPFN_PREC_BF16, fp32 for MMPFN_PREC_F32.  A query whose keys are all excluded gets 0.
 * Runs on the encoder's stream; needs no model. */
int mmpfn_enc_attention(mmpfn_enc* enc, const void* qkv, const float* kbias, void* out, int B, int L, int H,
                        int precision);

#ifdef __cplusplus
}
#endif

#endif /* MMPFN_MODALITY_H_ */
