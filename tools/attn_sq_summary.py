"""Summarise tools/attn_sq_pmc.sh: per-dispatch SQ / GRBM counters of the item-attention kernel (KSEL) (sums over
the kernel's dispatches divided by their count), plus derived ratios."""
import collections
import csv
import os
import sys
from pathlib import Path

root = Path(sys.argv[1])
acc = collections.defaultdict(float)
disp = collections.defaultdict(set)
for f in sorted(root.glob("*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if os.environ.get("KSEL", "attn_pipe") not in r["Kernel_Name"]:
            continue
        acc[r["Counter_Name"]] += float(r["Counter_Value"])
        disp[r["Counter_Name"]].add(r.get("Dispatch_Id", r.get("Correlation_Id")))
per = {k: v / max(1, len(disp[k])) for k, v in acc.items()}
for k in sorted(per):
    print(f"{k:28s} {per[k]:.4g}")
w = per.get("SQ_WAVE_CYCLES")
if w:
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_VALU",
              "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_MISC"):
        if k in per:
            print(f"{k}/SQ_WAVE_CYCLES = {per[k] / w:.3f}")
if "SQ_VALU_MFMA_BUSY_CYCLES" in per and "GRBM_GUI_ACTIVE" in per:
    # MFMA busy cycles summed over SIMDs vs the kernel's GPU-active cycles x 1024 SIMDs
    # (GRBM_GUI_ACTIVE is summed over the 8 XCDs: MI355X_MICROARCH.md DVFS note)
    act = per["GRBM_GUI_ACTIVE"] / 8
    print(f"MFMA pipe utilisation = {per['SQ_VALU_MFMA_BUSY_CYCLES'] / (act * 1024):.3f} of 1024 SIMDs x "
          f"{act:.4g} active cycles")
