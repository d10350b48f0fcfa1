"""Diagnostic (GPU): several MMPFNClassifier instances in one process, each timed over 10 predicts, round-robin twice;
prints each one's lane streams (HIP handles) -- why bench.py's api leg reads 13.2 or 15.2 ms per predict."""
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

cfg, sd, model, x, y, image, members = bench.build_workload(torch.device("cuda", 0), 1, 4)
X = x.astype(np.float64)
Xq, imq = X[1838:], image[1838:]
clfs = []
with tempfile.TemporaryDirectory() as tmp:
    ck = Path(tmp) / "c.ckpt"
    torch.save({"state_dict": {k: torch.from_numpy(v) for k, v in sd.items()}, "config": ckpt_config(cfg)}, ck)
    for i in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
        clf = MMPFNClassifier(model_path=str(ck), mixer_type="MGM+CAP", mgm_heads=64, cap_heads=24, features_per_group=2,
                              n_estimators=4, categorical_features_indices=list(range(18)), ignore_pretraining_limits=True,
                              inference_config=ModelInterfaceConfig(FINGERPRINT_FEATURE=False,
                                                                    PREPROCESS_TRANSFORMS=[PreprocessorConfig(name="none")]))
        clf.fit(X[:1838], image[:1838], y[:1838].astype(np.int64))
        for _ in range(3):
            clf.predict_proba(Xq, imq)
        clfs.append(clf)
print("MMPFN_LANE_STREAMS", __import__("os").environ.get("MMPFN_LANE_STREAMS", "pool"))
for r in range(2):
    for i, clf in enumerate(clfs):
        for _ in range(2):
            clf.predict_proba(Xq, imq)
        t0 = time.perf_counter()
        for _ in range(10):
            clf.predict_proba(Xq, imq)
        eng = clf.model_.engine(clf.device_)
        st = [hex(s.cuda_stream) for s in eng._streams]
        print(f"round {r} classifier {i}: {(time.perf_counter() - t0) * 100:.3f} ms per predict, lanes {st}", flush=True)
