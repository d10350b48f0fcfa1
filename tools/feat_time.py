"""Time the feature-attention sublayer kernel of the library named by MMPFN_LIB (one bf16 layer
of the config-C geometry through mmpfn_run_layers would include other kernels; this drives
the whole forward and reports rocprof-free per-layer wall time of the engine).
Usage: MMPFN_LIB=path python3 tools/feat_time.py"""
import os
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "tests" / "golden"))
import tools_prof_forward  # noqa: E402

t0 = time.time()
sys.argv = [sys.argv[0], "6"]
tools_prof_forward.main()
print(os.path.basename(os.environ.get("MMPFN_LIB", "default")), "wall", round(time.time() - t0, 2))
