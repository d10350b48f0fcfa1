"""Generate the modality-encoder golden vectors by running the REFERENCE towers (build container only).

Run from the repo root:   python tests/golden/make_modality_golden.py

* image: the reference's own DINOv2 code, imported read-only from /root/reference
  (mmpfn/models/dino_v2/models/vision_transformer.py ``DinoVisionTransformer`` built as ``vit_base``
  builds it: ``block_fn=partial(Block, attn_class=MemEffAttention)``, mlp_ratio 4, block_chunks 0,
  num_register_tokens 0; xFormers absent, so Attention uses torch SDPA), called as the dataset code
  calls it: ``forward_features(batch)["x_norm_clstoken"]`` (pad_ufes_20.py:95-96).
* text: transformers' ``ElectraModel`` (the model the reference loads by name, petfinder.py:155-178;
  transformers 5.15.0 in this container, the reference pins none), one text per call as the
  reference does; the masked case also runs the padded batch under ``attention_mask``.

Weights and inputs come from tests/golden/modality_cases.py (seeded); the outputs go to
tests/golden/modality_<case>.npz.  The reference never travels to the GPU box.
"""

from __future__ import annotations

import sys
from functools import partial
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))
from modality_cases import TEXT_CASES, VIT_CASES, text_config, text_inputs, text_state, vit_images, vit_state  # noqa: E402


def reference_vit(c: dict):
    sys.path.insert(0, "/root/reference")
    from mmpfn.models.dino_v2.layers import MemEffAttention, NestedTensorBlock as Block
    from mmpfn.models.dino_v2.models.vision_transformer import DinoVisionTransformer

    m = DinoVisionTransformer(img_size=c["img_size"], patch_size=c["patch"], embed_dim=c["dim"], depth=c["depth"],
                              num_heads=c["heads"], mlp_ratio=4, block_fn=partial(Block, attn_class=MemEffAttention),
                              num_register_tokens=0, init_values=c["init_values"], block_chunks=0,
                              interpolate_offset=c["offset"])
    sd = {k: torch.from_numpy(v) for k, v in vit_state(c).items()}
    m.load_state_dict(sd, strict=True)
    return m.eval()


def main() -> None:
    torch.set_num_threads(8)
    for name, c in VIT_CASES.items():
        m = reference_vit(c)
        x = torch.from_numpy(vit_images(c))
        with torch.no_grad():
            out = m.forward_features(x)
        cls = out["x_norm_clstoken"].numpy()
        tok = out["x_norm_patchtokens"].numpy()
        keep = min(tok.shape[1], 48)  # the first patch tokens (x_norm of every token is tested through them)
        np.savez_compressed(HERE / f"modality_{name}.npz", cls=cls, patch_tokens=tok[:, :keep],
                            input_sum=np.float64(x.double().sum()))
        print(name, cls.shape, tok.shape, float(np.abs(cls).max()))

    from transformers import ElectraConfig, ElectraModel

    for name, c in TEXT_CASES.items():
        m = ElectraModel(ElectraConfig(**text_config(c))).eval()
        sd = {k: torch.from_numpy(v) for k, v in text_state(c).items()}
        missing, unexpected = m.load_state_dict(sd, strict=False)
        assert not unexpected and all(k.endswith(("position_ids", "token_type_ids")) for k in missing), (missing, unexpected)
        ids, types = text_inputs(c)
        res = {}
        with torch.no_grad():
            for j, (t, tt) in enumerate(zip(ids, types)):  # one text per call, like petfinder.py:174-177
                h = m(input_ids=torch.from_numpy(t)[None], attention_mask=torch.ones(1, len(t), dtype=torch.long),
                      token_type_ids=torch.from_numpy(tt)[None]).last_hidden_state
                res[f"hidden_{j}"] = h[0].numpy()
            L = max(len(t) for t in ids)
            bid = np.zeros((len(ids), L), np.int64)
            bmask = np.zeros((len(ids), L), np.int64)
            btt = np.zeros((len(ids), L), np.int64)
            for j, (t, tt) in enumerate(zip(ids, types)):
                bid[j, :len(t)], bmask[j, :len(t)], btt[j, :len(t)] = t, 1, tt
            hb = m(input_ids=torch.from_numpy(bid), attention_mask=torch.from_numpy(bmask),
                   token_type_ids=torch.from_numpy(btt)).last_hidden_state
            res["batched_hidden"] = hb.numpy()
        np.savez_compressed(HERE / f"modality_{name}.npz", **res)
        print(name, {k: v.shape for k, v in res.items()})


if __name__ == "__main__":
    main()
