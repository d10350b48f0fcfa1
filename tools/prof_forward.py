"""Profiling driver: a few member forwards at the config-C shape (for rocprofv3 --pmc passes); MMPFN_PROF_PREC:
f16 (default, the fp16 mode), bf16, or f32 (the parity mode).

Usage (on the GPU box):  rocprofv3 --pmc <counters> -d <dir> -o run --output-format csv -- \
                              python3 tools/prof_forward.py [n_forwards]
"""

import os
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests" / "golden"))

from synth import synth_image, synth_labels, synth_state_dict, synth_table  # noqa: E402

from multimodalpfn_amd import _lib  # noqa: E402
from multimodalpfn_amd.model.spec import ModelConfig, state_dict_spec  # noqa: E402
from multimodalpfn_amd.model.transformer import PerFeatureTransformer  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    cfg = ModelConfig(mgm_heads=64, cap_heads=24)
    sd = synth_state_dict(state_dict_spec(cfg), 2)
    model = PerFeatureTransformer(cfg)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    model.to("cuda")
    eng = model.engine()
    S, N = 2298, 1838
    x = torch.from_numpy(synth_table(S, 21, 2, n_cat=18)).cuda()
    im = torch.from_numpy(synth_image(S, 1, 2)).cuda()
    y = synth_labels(S, 6, 2)[:N]
    prec = {"f32": _lib.PREC_F32, "bf16": _lib.PREC_BF16}.get(os.environ.get("MMPFN_PROF_PREC", "f16"), _lib.PREC_F16)
    tok = eng.mixer_tokens(im, prec)
    batch = int(os.environ.get("MMPFN_PROF_BATCH", "1"))  # members per batched forward
    for _ in range(n):
        if batch > 1:
            out = eng.forward_batch([(x, tok, y)] * batch, prec)[0]
        else:
            out = eng.forward(x, tok, y, prec, check_nan=False)
    eng.status()
    torch.cuda.synchronize()
    print("ok", tuple(out.shape), float(out.abs().mean()))


if __name__ == "__main__":
    main()
