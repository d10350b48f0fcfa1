#!/bin/bash
# round 6 GPU pass: smoke, the GPU test suite (its tail carries the measured numbers: conftest terminal summary), the
# 1-GPU bench, the one-lane kernel trace.  $1: output tag
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { tail -40 $O/pytest_gpu.log; exit 1; }
grep -E "passed|failed" $O/pytest_gpu.log | tail -1
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
tail -n 1 $O/bench.json | head -c 300; echo
[ "$2" = noprof ] || bash tools/prof_lanes1.sh ${1}_f16
