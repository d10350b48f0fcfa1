"""Diagnostic (GPU): bench.py's api_end_to_end leg in a fresh process, optionally after a headline-like engine has run
(`with-engine`: the bench's own HipEngine built and stepped first, as in bench.main)."""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "tests" / "golden")]
import bench  # noqa: E402
from multimodalpfn_amd import _lib  # noqa: E402

dev = torch.device("cuda", 0)
cfg, sd, model, x, y, image, members = bench.build_workload(dev, 1, 4)
if "with-engine" in sys.argv[1:]:
    eng = model.engine(dev)
    img = torch.from_numpy(image).to(dev)
    prec = _lib.PREC_F16
    import numpy as np
    step = bench.make_step(eng, members, list(range(4)), [list(range(4))], 0, img, prec, None, None)
    print("headline ms", bench.timed_steps(step, 30, 5, 1, dev) / 30 * 1e3)
for _ in range(2):
    r = bench.api_end_to_end(cfg, sd, x, y, image, 4, False, 10, 1)
    print("api ms per predict", r["ms_per_predict"])
