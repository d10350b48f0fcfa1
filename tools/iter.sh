#!/bin/bash
# Quick GPU iteration: selected parity tests (-k $K), then a short bench (no CPU/API legs).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread ${K:+-k "$K"} > gpurun_out/iter_pytest.log 2>&1
rc=$?
tail -5 gpurun_out/iter_pytest.log
case $rc in 0|1|5) ;; *) exit $rc ;; esac
[ $rc = 1 ] && exit 1
timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --api-steps 0 > gpurun_out/iter_bench.json 2> gpurun_out/iter_bench.err || { tail -20 gpurun_out/iter_bench.err; exit 1; }
cat gpurun_out/iter_bench.json
