"""Diagnostic (GPU): does a forward depend on what an earlier forward of another geometry left in
the lane workspace?  Member A alone on a fresh engine, then after member B (wider table), compared
tap by tap (embedded state, every layer, logits)."""
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "tests" / "golden"), str(ROOT / "tests")]
from synth import synth_image, synth_labels, synth_state_dict, synth_table  # noqa: E402

from multimodalpfn_amd import _lib  # noqa: E402
from multimodalpfn_amd.model.spec import ModelConfig, state_dict_spec  # noqa: E402
from multimodalpfn_amd.model.transformer import PerFeatureTransformer  # noqa: E402

S, N = int(sys.argv[1]) if len(sys.argv) > 1 else 2298, 1838
N = min(N, S - 100)
FA, FB = 21, int(sys.argv[2]) if len(sys.argv) > 2 else 51
cfg = ModelConfig(mgm_heads=64, cap_heads=24)
model = PerFeatureTransformer(cfg)
model.load_state_dict({k: torch.from_numpy(v) for k, v in synth_state_dict(state_dict_spec(cfg), 3).items()})
model.to("cuda")
eng = model.engine()
P = _lib.PREC_BF16
im = torch.from_numpy(synth_image(S, 2, 3)).cuda()
base = synth_table(S, 51, 3, n_cat=18)
xa = torch.from_numpy(np.ascontiguousarray(base[:, :FA])).cuda()
xb = torch.from_numpy(np.ascontiguousarray(base[:, :FB])).cuda()
y = synth_labels(S, 6, 3)[:N]


def taps(x, tok):
    out = [eng.embed_state(x, tok, y, P).cpu()]
    for l in range(cfg.nlayers):
        out.append(eng.run_layers(l, l + 1).cpu())
    return out


with torch.inference_mode():
    tok = eng.mixer_tokens(im, P)
    la = eng.forward(xa, tok, y, P).cpu()
    ta = taps(xa, tok)
    eng.forward(xb, tok, y, P)
    torch.cuda.synchronize()
    lb = eng.forward(xa, tok, y, P).cpu()
    tb = taps(xa, tok)
    eng.status()
print("logits fresh vs after B: maxdiff", (la - lb).abs().max().item())
for i, (a, b) in enumerate(zip(ta, tb)):
    d = (a - b).abs()
    name = "embed" if i == 0 else f"layer{i - 1}"
    bad = (d > 0).nonzero()
    print(f"{name}: maxdiff {d.max().item():.3e}  n_diff {int((d > 0).sum())}"
          + (f"  first at [s,t,e]={bad[0].tolist()} rows {sorted(set(bad[:, 0].tolist()))[:8]} "
             f"tokens {sorted(set(bad[:, 1].tolist()))[:12]}" if len(bad) else ""))

# batched (M = 2) vs single, and lanes, at this size
rng = np.random.default_rng(1)
xa2 = torch.from_numpy(np.ascontiguousarray(base[:, rng.permutation(51)[:FA]])).cuda()
y2 = rng.permutation(6)[y.astype(np.int64)].astype(np.float32)
with torch.inference_mode():
    s1 = eng.forward(xa, tok, y, P).cpu()
    s2 = eng.forward(xa2, tok, y2, P).cpu()
    b1, b2 = [o.cpu() for o in eng.forward_batch([(xa, tok, y), (xa2, tok, y2)], P)]
    m1, m2 = [o.cpu() for o in eng.forward_many([(xa, tok, y), (xa2, tok, y2)], P, lanes=2, batch=1)]
    eng.status()
print("batch M=2 vs single:", (b1 - s1).abs().max().item(), (b2 - s2).abs().max().item())
print("lanes=2 vs single:", (m1 - s1).abs().max().item(), (m2 - s2).abs().max().item())
