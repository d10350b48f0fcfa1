"""Parity mode (PREC_F32): logits error of the item attention's cheap form (fp16 S, two-product P.V)
against the key count N, on the golden models (their configs and synthetic weights) with synthetic inputs of N train
+ Q test rows.  Both item-attention forms run on the same inputs; the checker is the oracle evaluated in fp32 on the
GPU (pinned on CPU by the reference goldens).  The smallest N from which every model stays >= 2x under the 1e-4
contract picks the launcher's threshold (X3_CHEAP_MIN_KEYS, mmpfn_set_parity_attention_min_keys).

    python tools/parity_n0_sweep.py [N,N,...] [form] > profiles/r06/parity_n0_sweep_form<form>.txt
"""

from __future__ import annotations

import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "tests"), str(ROOT / "tests" / "golden")]

from helpers import CASES, load_case, oracle_spec, rel_err, torch_sd  # noqa: E402
from synth import synth_image, synth_labels, synth_table  # noqa: E402

from multimodalpfn_amd import _lib  # noqa: E402
from oracle.forward import oracle_forward  # noqa: E402

NS = [int(a) for a in sys.argv[1].split(",")] if len(sys.argv) > 1 and sys.argv[1] else [40, 64, 96, 128, 192, 256, 384, 512, 768,
                                                                          1024, 1536, 1838]
Q = 64
FORM = int(sys.argv[2]) if len(sys.argv) > 2 else 3  # attn_item3_kernel CHEAP bits: 1 fp16 S, 2 two-product P.V
DEFAULT_FORM = 3


def main():
    from test_parity_gpu import make_model

    lib = _lib.load_library()
    torch.backends.cuda.matmul.allow_tf32 = False
    print(f"# parity-mode item attention: cheap form {FORM} (bit 0 fp16 S, bit 1 two-product P.V) vs three products, logits rel err vs the "
          f"fp32 oracle on device; Q = {Q} test rows; columns: case, N, err_exact, err_cheap, ratio")
    worst: dict[int, float] = {}
    t0 = time.time()
    for case in CASES:
        z, meta, cfg, sd = load_case(case)
        F = z["x"].shape[1] if "x" in z else 0
        n_mod = z["image"].shape[1] if "image" in z else 0
        ncls = int(meta.get("n_classes", 3))
        data = dict(meta.get("data", {}))
        model = make_model(cfg, sd)
        w = {k: v.cuda() for k, v in torch_sd(sd).items()}
        for N in NS:
            S = N + Q
            seed = 1000 + N
            x = torch.from_numpy(synth_table(S, F, seed, n_cat=int(data.get("n_cat", 0)),
                                             nan_frac=float(data.get("nan_frac", 0.0)))).cuda() if F else None
            im = torch.from_numpy(synth_image(S, n_mod, seed)).cuda() if n_mod else None
            y = torch.from_numpy(synth_labels(S, ncls, seed)[:N]).cuda()
            outs = {}
            with torch.inference_mode():
                for name, mk in (("exact", -1), ("cheap", 0)):
                    prev = lib.mmpfn_set_parity_attention_min_keys(mk, FORM)
                    try:
                        outs[name] = model(None, x[:, None, :] if x is not None else None, im, y,
                                           single_eval_pos=N).squeeze(1).float().cpu().numpy()
                    finally:
                        lib.mmpfn_set_parity_attention_min_keys(prev, DEFAULT_FORM)
                ref = oracle_forward(oracle_spec(cfg), w, x, im, y).cpu().numpy()
            ee, ec = rel_err(outs["exact"], ref), rel_err(outs["cheap"], ref)
            worst[N] = max(worst.get(N, 0.0), ec)
            print(f"{case:14s} N={N:5d} exact {ee:.3e} cheap {ec:.3e} ratio {ec / max(ee, 1e-12):6.2f}", flush=True)
        del w, model
        torch.cuda.empty_cache()
    print("# worst cheap-form error per N over the models:")
    for N in NS:
        print(f"#   N={N:5d} {worst[N]:.3e} {'<= 5e-5 (2x under 1e-4)' if worst[N] <= 5e-5 else ''}")
    ok = [N for N in NS if all(worst[M] <= 5e-5 for M in NS if M >= N)]
    print(json.dumps({"n0_candidates": ok, "worst": worst, "seconds": round(time.time() - t0, 1)}))


if __name__ == "__main__":
    main()
