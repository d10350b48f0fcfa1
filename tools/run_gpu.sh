#!/bin/bash
# GPU session script: parity tests, bench, rocprof kernel stats (each step time-bounded).
set -o pipefail
R=$PWD
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest_rc=$rc" >> gpurun_out/pytest_gpu.log
tail -3 gpurun_out/pytest_gpu.log
# a crash / abort / time limit means the GPU may be unhealthy: stop here
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
cat gpurun_out/bench.json
export TMPDIR=/tmp
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $R/gpurun_out/bench_prof.json 2> $R/gpurun_out/bench_prof.err
