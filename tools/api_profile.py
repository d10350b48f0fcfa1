"""Diagnostic (GPU): where predict_proba's host time goes at config C (cProfile over 10 calls; `default`: the
reference's default member preprocessing)."""
import cProfile
import pstats
import sys
import tempfile
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

cfg, sd, model, x, y, image, members = bench.build_workload(torch.device("cuda", 0), 1, 4)
with tempfile.TemporaryDirectory() as tmp:
    ck = Path(tmp) / "c.ckpt"
    torch.save({"state_dict": {k: torch.from_numpy(v) for k, v in sd.items()}, "config": ckpt_config(cfg)}, ck)
    clf = MMPFNClassifier(model_path=str(ck), mixer_type="MGM+CAP", mgm_heads=64, cap_heads=24, features_per_group=2,
                          n_estimators=4, categorical_features_indices=list(range(18)), ignore_pretraining_limits=True,
                          inference_config=(ModelInterfaceConfig() if "default" in sys.argv[1:] else
                                            ModelInterfaceConfig(FINGERPRINT_FEATURE=False,
                                                                 PREPROCESS_TRANSFORMS=[PreprocessorConfig(name="none")])))
    X = x.astype(np.float64)
    clf.fit(X[:1838], image[:1838], y[:1838].astype(np.int64))
Xq, imq = X[1838:], image[1838:]
for _ in range(3):
    clf.predict_proba(Xq, imq)
import time  # noqa: E402
t0 = time.perf_counter()
for _ in range(10):
    clf.predict_proba(Xq, imq)
print("ms per predict", (time.perf_counter() - t0) * 100)
pr = cProfile.Profile()
pr.enable()
for _ in range(10):
    clf.predict_proba(Xq, imq)
pr.disable()
pstats.Stats(pr).sort_stats("cumulative").print_stats(45)
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
