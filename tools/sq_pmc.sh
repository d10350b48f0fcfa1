#!/bin/bash
# SQ counters (one pass, <= 8 SQ) over one bf16 forward: per-kernel wave-cycle breakdown
set -o pipefail
R=$PWD; mkdir -p gpurun_out; export TMPDIR=/tmp
LIB=${1:-}
cd /tmp || exit 1
MMPFN_DIAGNOSTICS=1 MMPFN_LIB=$LIB timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_MFMA \
  -d $R/gpurun_out/sqpmc -o run --output-format csv -- python3 $R/tools/prof_forward.py 1 > $R/gpurun_out/sqpmc.log 2>&1 || exit 1
cd $R && python3 - <<'PY'
import csv, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float))
dur = collections.defaultdict(list)
for r in csv.DictReader(open("gpurun_out/sqpmc/run_counter_collection.csv")):
    k = r["Kernel_Name"].split("(")[0][-40:]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in acc.items():
    if c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) < 1e6: continue
    w = c["SQ_WAVE_CYCLES"]
    print(f"{k:42s} wave {w:.3g}  wait {c['SQ_WAIT_ANY']/w:.2f} waitinst {c['SQ_WAIT_INST_ANY']/w:.2f} (lds {c['SQ_WAIT_INST_LDS']/w:.2f}) active {c['SQ_ACTIVE_INST_ANY']/w:.2f}  mfma_busy {c['SQ_VALU_MFMA_BUSY_CYCLES']:.3g} busy {c['SQ_BUSY_CYCLES']:.3g} n_mfma {c['SQ_INSTS_MFMA']:.3g}")
PY
