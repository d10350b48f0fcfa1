"""Golden logits of the REFERENCE forward under its own fp16 autocast (build container only).

Run from the repo root:   python tests/golden/make_f16_golden.py [case ...]

The reference's GPU inference runs the model under ``torch.autocast(device, dtype=float16)``
(``utils.py:150-190`` -> ``inference.py:343-348``), with its LayerNorm kept in fp16 by ``layer.py:60-62``
(autocast disabled around ``layer_norm`` when the input is fp16).  Here the same reference model of every
``make_golden.py`` case (same synthetic weights and inputs) is called under ``torch.autocast("cpu",
dtype=torch.float16)``: ``layer.py:61`` picks ``"cpu"`` for CPU tensors, so its fp16 LayerNorm applies too.

CPU autocast differs from CUDA autocast in two places that touch this forward (both are recorded in DESIGN.md
section 3): without a visible GPU the reference takes its einsum-softmax attention branch
(``multi_head_attention.py:718-729``) instead of ``scaled_dot_product_attention`` (``:693-717``), and CPU
autocast keeps ``softmax`` / ``exp`` in fp16 where CUDA autocast promotes them to fp32.  Both round the
probabilities to fp16 before ``P.V``, as CUDA's fp16 SDPA kernels do.

Written to ``tests/golden/f16/<case>.npz``: ``logits_f16`` (the reference's fp16-autocast logits, as fp32) and
``logits_f32`` (the same reference model in fp32, equal to the case's ``logits`` in ``tests/golden/<case>.npz``
where that file exists).  ``logits_f16`` draws the positional embedding's random vectors in fp32 (see ``run``);
``logits_f16_f16draws`` is the unmodified fp16 run, whose fp16 draws are a different random stream.  The additional ``pad_ufes_c_reduced`` case is config C's model (12 layers, MGM 64 +
CAP 24, F = 21 with 18 categorical, 6 classes) on 600 rows; its inputs are stored in its own file.
"""

from __future__ import annotations

import os
import sys
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))

import make_golden as mg  # noqa: E402

EXTRA = [
    dict(name="pad_ufes_c_reduced", cfg=dict(nlayers=12, mgm_heads=64, cap_heads=24), S=600, N=480, F=21,
         data=dict(n_cat=18), n_mod=1, n_classes=6, wseed=2, dseed=109),
]


def run(case: dict, f16: bool, fp32_draws: bool = True) -> dict:
    """make_golden.run_case with the reference forward under CPU fp16 autocast when ``f16``.

    ``fp32_draws``: the subspace positional embedding's random vectors are drawn with ``dtype=x.dtype``
    (``transformer.py:921-926``), i.e. in fp16 under autocast -- a different random stream than the fp32 forward's,
    not a rounding of it.  With ``fp32_draws`` they are drawn in fp32 from the same generator and rounded to fp16,
    so the fp16 run differs from the fp32 run by its arithmetic alone."""
    if not f16:
        return mg.run_case(case)
    orig = torch.inference_mode
    orig_randn = torch.randn

    def randn_fp32_draws(*a, dtype=None, **k):
        if dtype == torch.float16:
            return orig_randn(*a, dtype=torch.float32, **k).to(torch.float16)
        return orig_randn(*a, dtype=dtype, **k)

    def autocast_inference_mode(*a, **k):  # run_case's forward runs inside torch.inference_mode()
        class Ctx:
            def __enter__(self):
                self.im = orig(*a, **k)
                self.ac = torch.autocast("cpu", dtype=torch.float16)
                self.im.__enter__()
                self.ac.__enter__()

            def __exit__(self, *exc):
                self.ac.__exit__(*exc)
                return self.im.__exit__(*exc)
        return Ctx()

    torch.inference_mode = autocast_inference_mode
    if fp32_draws:
        torch.randn = randn_fp32_draws
    try:
        return mg.run_case(case)
    finally:
        torch.inference_mode = orig
        torch.randn = orig_randn


def main():
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    only = set(sys.argv[1:])
    out_dir = HERE / "f16"
    out_dir.mkdir(exist_ok=True)
    for case in mg.CASES + EXTRA:
        if only and case["name"] not in only:
            continue
        case = {k: v for k, v in case.items() if k != "taps"}
        r32 = run(case, False)
        r16 = run(case, True)
        r16d = run(case, True, fp32_draws=False)
        res = {"logits_f16": r16["logits"].astype(np.float32), "logits_f32": r32["logits"],
               "logits_f16_f16draws": r16d["logits"].astype(np.float32)}
        if case in EXTRA:  # no make_golden file: keep the inputs here
            res.update({k: r32[k] for k in ("x", "image", "y_train", "meta") if k in r32})
        else:
            g = np.load(HERE / f"{case['name']}.npz")
            assert np.array_equal(g["logits"], r32["logits"]), case["name"]  # the same reference forward
        d = float(np.abs(res["logits_f16"] - res["logits_f32"]).max() / max(1.0, np.abs(res["logits_f32"]).max()))
        agree = float((res["logits_f16"].argmax(1) == res["logits_f32"].argmax(1)).mean())
        path = out_dir / f"{case['name']}.npz"
        np.savez_compressed(path, **res)
        dd = float(np.abs(res["logits_f16_f16draws"] - res["logits_f32"]).max() / max(1.0, np.abs(res["logits_f32"]).max()))
        print(f"{case['name']}: reference fp16 vs fp32 rel dev {d:.3e}, argmax agreement {agree:.4f} "
              f"(fp16 draws: {dd:.3e}) -> {path.name}")


if __name__ == "__main__":
    main()
