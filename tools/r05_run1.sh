#!/bin/bash
# round 5, first GPU pass: the GPU test suite, the 1-GPU bench, the launcher rehearsal
set -o pipefail
O=gpurun_out/r05a; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
tail -n 1 $O/bench.json | head -c 600; echo
bash tools/rehearse_multirank.sh
