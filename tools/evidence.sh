#!/bin/bash
# Round evidence on the GPU box: gpu parity tests, smoke, default bench line, rocprofv3 kernel
# trace + stats of the bench command (cpu leg skipped), summarised by launch grid.
# Each GPU step is time-bounded; the script stops at the first failure.
set -o pipefail
R=$PWD; TAG=${1:-run}; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cd /tmp || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/rprof -o run --output-format csv -- \
  python3 $R/bench.py --no-cpu-baseline > $O/bench_prof.json 2> $O/bench_prof.err || exit 1
cd $R && python3 tools/ktrace_grid.py $O/rprof/run_kernel_trace.csv 40 > $O/rprof_by_grid.txt
head -c 600 $O/bench.json
