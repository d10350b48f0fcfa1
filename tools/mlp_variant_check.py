"""The MLP sublayer of the selected kernel (MMPFN_MLP32=1: mlp32.hip, else mlp_rows.hip) against the oracle at the
config-C shape (S=2298, T=36: the plain tap and the fused out-projection form through a full bf16 forward), plus
the tap's kernel time.  Usage: [MMPFN_MLP32=1] python3 tools/mlp_variant_check.py"""
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
sys.path.insert(0, str(ROOT / "tests" / "golden"))
from helpers import oracle_spec, rel_err, torch_sd  # noqa: E402
from oracle.forward import mlp_sublayer, oracle_forward  # noqa: E402
from synth import synth_image, synth_labels, synth_state_dict, synth_table  # noqa: E402

from multimodalpfn_amd import _lib  # noqa: E402
from multimodalpfn_amd.model.spec import ModelConfig, state_dict_spec  # noqa: E402
from multimodalpfn_amd.model.transformer import PerFeatureTransformer  # noqa: E402

tag = "mlp32" if os.environ.get("MMPFN_MLP32") == "1" else "mlp_rows"
torch.backends.cuda.matmul.allow_tf32 = False
cfg = ModelConfig(mgm_heads=64, cap_heads=24)
sd = synth_state_dict(state_dict_spec(cfg), 2)
model = PerFeatureTransformer(cfg)
model.load_state_dict(torch_sd(sd))
norm = next(e for e in model.encoder if "InputNormalizationEncoderStep" in str(e.__class__))
norm.remove_outliers, norm.remove_outliers_sigma = True, 12.0
model.to("cuda")
eng = model.engine()
spec, w = oracle_spec(cfg), {k: v.cuda() for k, v in torch_sd(sd).items()}
g = torch.Generator(device="cpu").manual_seed(3)
X = torch.randn(2298, 36, 192, generator=g).cuda()
with torch.inference_mode():
    ref = mlp_sublayer(spec, w, 0, X)
    got = eng.mlp_ln(0, X, _lib.PREC_BF16)
    torch.cuda.synchronize()
    print(f"{tag}: mlp tap rel err {rel_err(got.cpu().numpy(), ref.cpu().numpy()):.3e}")
    Xd = X.reshape(-1, 192).contiguous()
    for _ in range(3):
        eng.mlp_ln(0, Xd, _lib.PREC_BF16)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        eng.mlp_ln(0, Xd, _lib.PREC_BF16)
    torch.cuda.synchronize()
    print(f"{tag}: mlp tap (one member, plain) {(time.perf_counter() - t0) / 20 * 1e6:.1f} us per call incl. copies")
    S, N = 2298, 1838
    x = torch.from_numpy(synth_table(S, 21, 2, n_cat=18)).cuda()
    im = torch.from_numpy(synth_image(S, 1, 2)).cuda()
    y = torch.from_numpy(synth_labels(S, 6, 2)[:N]).cuda()
    with torch.autocast("cuda"):
        b16 = model(None, x[:, None, :], im, y, single_eval_pos=N).squeeze(1).float().cpu().numpy()
    refl = oracle_forward(spec, w, x, im, y).cpu().numpy()
    agree = float((b16.argmax(1) == refl.argmax(1)).mean())
    print(f"{tag}: config-C bf16 logits rel err {rel_err(b16, refl):.3e}, argmax agreement {agree:.4f}")
