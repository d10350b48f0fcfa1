#!/bin/bash
# round-5 final evidence: GPU suite, smoke, numbers, bench (+ launcher rehearsal), one-lane kernel trace
set -o pipefail
O=gpurun_out/${1:-r05z}; mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash tools/r05_run.sh ${1:-r05z} || exit 1
bash tools/prof_lanes1.sh ${1:-r05z}_f16 || exit 1
