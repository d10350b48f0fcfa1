"""Diagnostic (GPU): config-D ragged members through forward_many under several schedules vs
single forwards; prints the per-member max |diff|."""
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "tests" / "golden"), str(ROOT / "tests")]
from synth import synth_image, synth_state_dict  # noqa: E402
from test_configs_gpu import _ragged_members, S_ROWS  # noqa: E402

from multimodalpfn_amd import _lib  # noqa: E402
from multimodalpfn_amd.model.spec import ModelConfig, state_dict_spec  # noqa: E402
from multimodalpfn_amd.model.transformer import PerFeatureTransformer  # noqa: E402

cfg = ModelConfig(mgm_heads=64, cap_heads=24)
model = PerFeatureTransformer(cfg)
model.load_state_dict({k: torch.from_numpy(v) for k, v in synth_state_dict(state_dict_spec(cfg), 3).items()})
model.to("cuda")
eng = model.engine()
P = _lib.PREC_BF16
n = int(sys.argv[1]) if len(sys.argv) > 1 else 32
with torch.inference_mode():
    im = torch.from_numpy(synth_image(S_ROWS, 2, 3)).cuda()
    tok = eng.mixer_tokens(im, P)
    items = [(xm.cuda(), tok, ym) for xm, ym in _ragged_members(n, 3, None)]
    single = [eng.forward(x, t, y, P).cpu() for x, t, y in items]
    for lanes, batch in [(1, 1), (1, 2), (2, 1), (2, 2), (2, 2)]:
        outs = [o.cpu() for o in eng.forward_many(items, P, lanes=lanes, batch=batch)]
        eng.status()
        d = [float((a - b).abs().max()) for a, b in zip(outs, single)]
        print(f"lanes {lanes} batch {batch}: max {max(d):.2e} bad members {[i for i, v in enumerate(d) if v > 0]}")
# same-geometry members only (all F = 21)
with torch.inference_mode():
    same = [it for it in items if it[0].shape[1] == 21] * 2
    single_s = [eng.forward(x, t, y, P).cpu() for x, t, y in same]
    outs = [o.cpu() for o in eng.forward_many(same, P, lanes=2, batch=1)]
    eng.status()
    d = [float((a - b).abs().max()) for a, b in zip(outs, single_s)]
    print(f"same-geometry lanes 2: max {max(d):.2e} bad {[i for i, v in enumerate(d) if v > 0]}")
