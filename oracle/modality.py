"""CPU oracle of the modality encoders -- TEST INFRASTRUCTURE ONLY.

Plain-torch fp32 restatement of the two towers whose outputs the reference caches as its image /
text tokens, written from the reference's code, one function per step:

* DINOv2 ``DinoVisionTransformer.forward_features`` (mmpfn/models/dino_v2/models/vision_transformer.py:
  180-212 interpolate_pos_encoding, :214-233 prepare_tokens_with_masks, :255-271 forward_features;
  layers/patch_embed.py PatchEmbed = Conv2d(kernel = stride = patch) + flatten; layers/block.py:93-130
  Block.forward ``x + ls1(attn(norm1(x)))``, ``x + ls2(mlp(norm2(x)))``; layers/attention.py:58-77
  qkv -> SDPA (scale head_dim**-0.5) -> proj; layers/mlp.py fc1 -> GELU -> fc2; LayerNorm eps 1e-6).
* transformers ``ElectraModel`` (the reference loads google/electra-base-discriminator by name,
  petfinder.py:155-178; third-party, transformers 5.15.0 here, the reference pins none):
  ElectraEmbeddings ``LN((word + type) + pos)``, optional ``embeddings_project``, BERT layers
  ``LN1(x + dense(attn(x)))``, ``LN2(x + out(gelu(inter(x))))`` with the additive attention mask.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s CPU-baseline leg may use this module;
the product path (multimodalpfn_amd.modality) never imports it.  Pinned by golden vectors made by
running the reference's own ``vit_base`` and transformers' ``ElectraModel`` on seeded random weights
(tests/golden/make_modality_golden.py).
"""

from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def interpolate_pos(pos_embed: torch.Tensor, gh: int, gw: int, offset: float = 0.1) -> torch.Tensor:
    """interpolate_pos_encoding (vision_transformer.py:180-212) for a (gh, gw) patch grid."""
    N = pos_embed.shape[1] - 1
    M = int(math.sqrt(N))
    if gh == M and gw == M:
        return pos_embed
    pe = pos_embed.float()
    cls, patch = pe[:, 0], pe[:, 1:]
    dim = pe.shape[-1]
    if offset:
        kw = {"scale_factor": (float(gh + offset) / M, float(gw + offset) / M)}
    else:
        kw = {"size": (gh, gw)}
    patch = F.interpolate(patch.reshape(1, M, M, dim).permute(0, 3, 1, 2), mode="bicubic", antialias=False, **kw)
    assert patch.shape[-2:] == (gh, gw)
    patch = patch.permute(0, 2, 3, 1).reshape(1, -1, dim)
    return torch.cat((cls.unsqueeze(0), patch), dim=1)


def vit_forward_features(sd: dict, x: torch.Tensor, *, patch: int, heads: int, depth: int, eps: float = 1e-6,
                         offset: float = 0.1, layerscale: bool = True) -> dict:
    """forward_features -> {"x_norm_clstoken", "x_norm_patchtokens", "x_prenorm"} (fp32, CPU)."""
    B, C, H, W = x.shape
    t = F.conv2d(x, sd["patch_embed.proj.weight"], sd["patch_embed.proj.bias"], stride=patch)  # PatchEmbed
    t = t.flatten(2).transpose(1, 2)
    t = torch.cat((sd["cls_token"].expand(B, -1, -1), t), dim=1)
    t = t + interpolate_pos(sd["pos_embed"], H // patch, W // patch, offset)
    D = t.shape[-1]
    for i in range(depth):
        p = f"blocks.{i}."
        h = F.layer_norm(t, (D,), sd[p + "norm1.weight"], sd[p + "norm1.bias"], eps)
        qkv = F.linear(h, sd[p + "attn.qkv.weight"], sd[p + "attn.qkv.bias"]).reshape(B, -1, 3, heads, D // heads)
        q, k, v = [u.transpose(1, 2) for u in torch.unbind(qkv, 2)]
        a = F.scaled_dot_product_attention(q, k, v).transpose(1, 2).reshape(B, -1, D)
        a = F.linear(a, sd[p + "attn.proj.weight"], sd[p + "attn.proj.bias"])
        t = t + (a * sd[p + "ls1.gamma"] if layerscale else a)
        h = F.layer_norm(t, (D,), sd[p + "norm2.weight"], sd[p + "norm2.bias"], eps)
        h = F.linear(F.gelu(F.linear(h, sd[p + "mlp.fc1.weight"], sd[p + "mlp.fc1.bias"])),
                     sd[p + "mlp.fc2.weight"], sd[p + "mlp.fc2.bias"])
        t = t + (h * sd[p + "ls2.gamma"] if layerscale else h)
    xn = F.layer_norm(t, (D,), sd["norm.weight"], sd["norm.bias"], eps)
    return {"x_norm_clstoken": xn[:, 0], "x_norm_patchtokens": xn[:, 1:], "x_prenorm": t}


def electra_forward(sd: dict, input_ids: torch.Tensor, attention_mask: torch.Tensor | None = None,
                    token_type_ids: torch.Tensor | None = None, *, heads: int, depth: int,
                    eps: float = 1e-12) -> torch.Tensor:
    """ElectraModel(...).last_hidden_state (fp32, CPU)."""
    B, L = input_ids.shape
    if token_type_ids is None:
        token_type_ids = torch.zeros_like(input_ids)
    e = sd["embeddings.word_embeddings.weight"][input_ids] + sd["embeddings.token_type_embeddings.weight"][token_type_ids]
    e = e + sd["embeddings.position_embeddings.weight"][torch.arange(L)][None]
    E = e.shape[-1]
    x = F.layer_norm(e, (E,), sd["embeddings.LayerNorm.weight"], sd["embeddings.LayerNorm.bias"], eps)
    if "embeddings_project.weight" in sd:
        x = F.linear(x, sd["embeddings_project.weight"], sd["embeddings_project.bias"])
    D = x.shape[-1]
    bias = None
    if attention_mask is not None:  # extended mask: (1 - m) * finfo.min, added to the scores
        bias = (1.0 - attention_mask[:, None, None, :].float()) * torch.finfo(torch.float32).min
    for i in range(depth):
        p = f"encoder.layer.{i}."
        def proj(name, t):
            return F.linear(t, sd[p + name + ".weight"], sd[p + name + ".bias"])
        q = proj("attention.self.query", x).reshape(B, L, heads, -1).transpose(1, 2)
        k = proj("attention.self.key", x).reshape(B, L, heads, -1).transpose(1, 2)
        v = proj("attention.self.value", x).reshape(B, L, heads, -1).transpose(1, 2)
        s = q @ k.transpose(-1, -2) * (q.shape[-1] ** -0.5)
        if bias is not None:
            s = s + bias
        a = (torch.softmax(s, -1) @ v).transpose(1, 2).reshape(B, L, D)
        x = F.layer_norm(x + proj("attention.output.dense", a), (D,), sd[p + "attention.output.LayerNorm.weight"],
                         sd[p + "attention.output.LayerNorm.bias"], eps)
        h = proj("output.dense", F.gelu(proj("intermediate.dense", x)))
        x = F.layer_norm(x + h, (D,), sd[p + "output.LayerNorm.weight"], sd[p + "output.LayerNorm.bias"], eps)
    return x
