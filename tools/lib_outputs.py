"""Diagnostics: the fp16- and bf16-mode logits of every golden case under one engine library (MMPFN_LIB), saved to
an .npz, so that two builds meant to be bitwise equal can be compared:  MMPFN_LIB=... python tools/lib_outputs.py out.npz
then  python tools/lib_outputs.py --compare a.npz b.npz"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tests"), str(ROOT / "tests" / "golden")]


def main():
    if sys.argv[1] == "--compare":
        a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
        bad = [k for k in a.files if not np.array_equal(a[k], b[k])]
        for k in a.files:
            print(f"{k}: {'EQUAL' if k not in bad else 'DIFF max %.3e' % np.abs(a[k] - b[k]).max()}")
        sys.exit(1 if bad else 0)
    from helpers import CASES, load_case
    from test_parity_gpu import make_model, run_case

    from multimodalpfn_amd import _lib

    res = {}
    for case in CASES:
        z, meta, cfg, sd = load_case(case)
        model = make_model(cfg, sd)
        for name, p in (("f16", _lib.PREC_F16), ("bf16", _lib.PREC_BF16)):
            res[f"{case}_{name}"] = run_case(z, model, precision=p)
    np.savez(sys.argv[1], **res)
    print("saved", len(res), "outputs to", sys.argv[1])


if __name__ == "__main__":
    main()
