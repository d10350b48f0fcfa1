"""A/B (GPU): predict_proba wall time at config C (bench.py's api leg, run.py's interface config) under two values of
an environment switch read per call, interleaved in rounds of 10 predicts.

    python tools/api_ab.py MMPFN_LANE_START eager together [rounds]
"""
import os
import sys
import tempfile
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "tests" / "golden")]
import bench  # noqa: E402
from api_cases import ckpt_config  # noqa: E402

from multimodalpfn_amd import MMPFNClassifier  # noqa: E402
from multimodalpfn_amd.constants import ModelInterfaceConfig  # noqa: E402
from multimodalpfn_amd.preprocessing import PreprocessorConfig  # noqa: E402

var, vals = sys.argv[1], sys.argv[2:4]
rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 4
default = "default" in sys.argv[5:]
cfg, sd, model, x, y, image, members = bench.build_workload(torch.device("cuda", 0), 1, 4)
with tempfile.TemporaryDirectory() as tmp:
    ck = Path(tmp) / "c.ckpt"
    torch.save({"state_dict": {k: torch.from_numpy(v) for k, v in sd.items()}, "config": ckpt_config(cfg)}, ck)
    clf = MMPFNClassifier(model_path=str(ck), mixer_type="MGM+CAP", mgm_heads=64, cap_heads=24, features_per_group=2,
                          n_estimators=4, categorical_features_indices=list(range(18)), ignore_pretraining_limits=True,
                          inference_config=(ModelInterfaceConfig() if default else
                                            ModelInterfaceConfig(FINGERPRINT_FEATURE=False,
                                                                 PREPROCESS_TRANSFORMS=[PreprocessorConfig(name="none")])))
    X = x.astype(np.float64)
    clf.fit(X[:1838], image[:1838], y[:1838].astype(np.int64))
Xq, imq = X[1838:], image[1838:]
ref = None
res = {v: [] for v in vals}
for r in range(rounds):
    for v in vals:
        os.environ[var] = v
        for _ in range(3):
            out = clf.predict_proba(Xq, imq)
        if ref is None:
            ref = out
        assert np.array_equal(out, ref), v
        t0 = time.perf_counter()
        for _ in range(10):
            clf.predict_proba(Xq, imq)
        res[v].append((time.perf_counter() - t0) * 100)
        print(f"round {r} {var}={v}: {res[v][-1]:.3f} ms per predict", flush=True)
for v in vals:
    print(f"{var}={v}: median {np.median(res[v]):.3f} ms per predict, all {[round(a, 3) for a in res[v]]}")
