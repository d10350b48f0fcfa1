"""Diagnostic (GPU): config-E logits (S = 12000, N = 10000, F = 20, tabular, 12 layers) from the
library named by MMPFN_LIB, in the bf16 mode and the fp32 parity mode; writes
gpurun_out/e_logits_<tag>.npz and prints the bf16 mode's deviation from the fp32 mode."""
import os
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "tests" / "golden")]
from synth import synth_labels, synth_state_dict, synth_table  # noqa: E402

from multimodalpfn_amd.model.spec import ModelConfig, state_dict_spec  # noqa: E402
from multimodalpfn_amd.model.transformer import PerFeatureTransformer  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else "main"
S, N, F, seed = 12000, 10000, 20, 4
cfg = ModelConfig(mgm_heads=8, cap_heads=4)
model = PerFeatureTransformer(cfg)
model.load_state_dict({k: torch.from_numpy(v) for k, v in synth_state_dict(state_dict_spec(cfg), seed).items()})
norm = next(e for e in model.encoder if "InputNormalizationEncoderStep" in str(e.__class__))
norm.remove_outliers, norm.remove_outliers_sigma = True, 12.0
model.to("cuda")
x = torch.from_numpy(synth_table(S, F, seed, nan_frac=0.01)).cuda()[:, None, :]
y = torch.from_numpy(synth_labels(S, 4, seed)[:N]).cuda()
with torch.inference_mode():
    f32 = model(None, x, None, y, single_eval_pos=N).squeeze(1).float().cpu().numpy()
    with torch.autocast("cuda"):
        b16 = model(None, x, None, y, single_eval_pos=N).squeeze(1).float().cpu().numpy()
os.makedirs("gpurun_out", exist_ok=True)
np.savez(f"gpurun_out/e_logits_{tag}.npz", f32=f32, b16=b16)
err = np.abs(b16 - f32).max() / max(1.0, np.abs(f32).max())
agree = (b16.argmax(1) == f32.argmax(1)).mean()
print(f"{tag}: config E perf-mode logits vs fp32 mode: rel err {err:.3e}, argmax agreement {agree:.4f}")
