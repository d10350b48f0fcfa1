#!/bin/bash
# HBM bytes per launch of every layer kernel (two rocprofv3 --pmc passes over batched bf16 forwards,
# MMPFN_PROF_BATCH=2 = the bench's launch shape): read = 2 x FETCH_SIZE (gfx950 correction), write =
# WRITE_SIZE, both in KB in the counter -> gpurun_out/<tag>/summary.txt
set -o pipefail
R=$PWD; TAG=${1:-lhbm}; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp MMPFN_PROF_BATCH=2
cd /tmp || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c -d $O/$c -o run --output-format csv -- python3 $R/tools/prof_forward.py 1 \
    > $O/$c.log 2>&1 || { tail -5 $O/$c.log; exit 1; }
done
cd $R && python3 - "$O" <<'PY' | tee $O/summary.txt
import csv, sys, collections
from pathlib import Path
o = Path(sys.argv[1]); acc = collections.defaultdict(lambda: collections.defaultdict(list))
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    for f in (o / c).rglob("*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            acc[r["Kernel_Name"][:48]][c].append(float(r["Counter_Value"]))
print(f"{'kernel':48s} {'n':>4s} {'read MB':>9s} {'write MB':>9s}")
for k, d in sorted(acc.items(), key=lambda kv: -sum(kv[1].get('FETCH_SIZE', [0]))):
    fe, wr = d.get("FETCH_SIZE", [0]), d.get("WRITE_SIZE", [0])
    print(f"{k:48s} {len(fe):4d} {2 * sum(fe) / len(fe) / 1024:9.1f} {sum(wr) / len(wr) / 1024:9.1f}")
PY
