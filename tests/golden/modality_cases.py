"""Seeded cases of the modality-encoder goldens (shared by make_modality_golden.py and the tests).

Weights are drawn from numpy PCG64 streams (O(1/sqrt(fan_in)) projections, perturbed LayerNorm and
LayerScale parameters), with the reference's state-dict names and shapes, so a test regenerates the
exact tensors the golden was made with and only the outputs need committing.
"""

from __future__ import annotations

import numpy as np

# ViT: the reference's vit_base geometry (embed 768, 12 heads, patch 14, pos grid of img_size 518)
VIT_CASES = {
    # two 56 x 56 images (4 x 4 patches): bicubic pos-embed resampling 37 -> 4 with offset 0.1
    "vit_small_img": dict(dim=768, depth=12, heads=12, patch=14, img_size=518, init_values=1.0, offset=0.1,
                          B=2, H=56, W=56, seed=11),
    # the reference's PAD-UFES resolution (img_size 14 * 24 = 336: 576 patches + CLS)
    "vit_336": dict(dim=768, depth=12, heads=12, patch=14, img_size=518, init_values=1.0, offset=0.1,
                    B=1, H=336, W=336, seed=12),
    # no LayerScale, interpolation to an exact size (offset 0), non-square 42 x 70 images, 2 blocks
    "vit_rect_nols": dict(dim=768, depth=2, heads=12, patch=14, img_size=518, init_values=None, offset=0.0,
                          B=3, H=42, W=70, seed=13),
}

# ELECTRA: google/electra-base-discriminator geometry; the reference tokenises and runs one text at a time
TEXT_CASES = {
    "electra_base": dict(vocab=30522, emb=768, dim=768, depth=12, heads=12, ffn=3072, max_pos=512, types=2,
                         lengths=[9, 23], seed=21),
    # embedding_size != hidden_size (embeddings_project), a padded batch under attention_mask
    "electra_proj_masked": dict(vocab=1000, emb=256, dim=768, depth=2, heads=12, ffn=1536, max_pos=64, types=2,
                                lengths=[5, 17, 12], seed=22),
}


def _rng(seed: int) -> np.random.Generator:
    return np.random.Generator(np.random.PCG64(seed))


def _lin(r, name, n_out, n_in, sd, bias=True):
    sd[name + ".weight"] = (r.standard_normal((n_out, n_in), dtype=np.float32) / np.float32(np.sqrt(n_in)))
    if bias:
        sd[name + ".bias"] = r.standard_normal(n_out, dtype=np.float32) * np.float32(0.05)


def _ln(r, name, n, sd):
    sd[name + ".weight"] = np.float32(1.0) + r.standard_normal(n, dtype=np.float32) * np.float32(0.1)
    sd[name + ".bias"] = r.standard_normal(n, dtype=np.float32) * np.float32(0.1)


def vit_state(c: dict) -> dict:
    r = _rng(c["seed"])
    D, P, G = c["dim"], c["patch"], c["img_size"] // c["patch"]
    sd = {}
    sd["cls_token"] = r.standard_normal((1, 1, D), dtype=np.float32)
    sd["pos_embed"] = r.standard_normal((1, 1 + G * G, D), dtype=np.float32) * np.float32(0.5)
    sd["mask_token"] = np.zeros((1, D), np.float32)
    sd["patch_embed.proj.weight"] = r.standard_normal((D, 3, P, P), dtype=np.float32) / np.float32(np.sqrt(3 * P * P))
    sd["patch_embed.proj.bias"] = r.standard_normal(D, dtype=np.float32) * np.float32(0.05)
    for i in range(c["depth"]):
        p = f"blocks.{i}."
        _ln(r, p + "norm1", D, sd)
        _lin(r, p + "attn.qkv", 3 * D, D, sd)
        _lin(r, p + "attn.proj", D, D, sd)
        _ln(r, p + "norm2", D, sd)
        _lin(r, p + "mlp.fc1", 4 * D, D, sd)
        _lin(r, p + "mlp.fc2", D, 4 * D, sd)
        if c["init_values"]:
            sd[p + "ls1.gamma"] = r.uniform(0.2, 1.0, D).astype(np.float32)
            sd[p + "ls2.gamma"] = r.uniform(0.2, 1.0, D).astype(np.float32)
    _ln(r, "norm", D, sd)
    return sd


def vit_images(c: dict) -> np.ndarray:
    r = _rng(c["seed"] + 1000)
    return r.uniform(0.0, 1.0, (c["B"], 3, c["H"], c["W"])).astype(np.float32)  # pixels / 255 like the dataset


def text_state(c: dict) -> dict:
    r = _rng(c["seed"])
    D, E = c["dim"], c["emb"]
    sd = {}
    sd["embeddings.word_embeddings.weight"] = r.standard_normal((c["vocab"], E), dtype=np.float32)
    sd["embeddings.position_embeddings.weight"] = r.standard_normal((c["max_pos"], E), dtype=np.float32) * np.float32(0.5)
    sd["embeddings.token_type_embeddings.weight"] = r.standard_normal((c["types"], E), dtype=np.float32) * np.float32(0.5)
    _ln(r, "embeddings.LayerNorm", E, sd)
    if E != D:
        _lin(r, "embeddings_project", D, E, sd)
    for i in range(c["depth"]):
        p = f"encoder.layer.{i}."
        _lin(r, p + "attention.self.query", D, D, sd)
        _lin(r, p + "attention.self.key", D, D, sd)
        _lin(r, p + "attention.self.value", D, D, sd)
        _lin(r, p + "attention.output.dense", D, D, sd)
        _ln(r, p + "attention.output.LayerNorm", D, sd)
        _lin(r, p + "intermediate.dense", c["ffn"], D, sd)
        _lin(r, p + "output.dense", D, c["ffn"], sd)
        _ln(r, p + "output.LayerNorm", D, sd)
    return sd


def text_inputs(c: dict):
    """Per-sequence token ids / token types (CLS-like id first; the second half of longer texts in segment 1)."""
    r = _rng(c["seed"] + 1000)
    ids, types = [], []
    for n in c["lengths"]:
        t = r.integers(1, c["vocab"], n).astype(np.int64)
        t[0] = min(101, c["vocab"] - 1)
        ids.append(t)
        tt = np.zeros(n, np.int64)
        if n > 10:
            tt[n // 2:] = 1
        types.append(tt)
    return ids, types


def text_config(c: dict) -> dict:
    return dict(vocab_size=c["vocab"], embedding_size=c["emb"], hidden_size=c["dim"], num_hidden_layers=c["depth"],
                num_attention_heads=c["heads"], intermediate_size=c["ffn"], max_position_embeddings=c["max_pos"],
                type_vocab_size=c["types"], hidden_act="gelu", layer_norm_eps=1e-12)
