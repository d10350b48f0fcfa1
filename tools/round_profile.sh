#!/bin/bash
# Round-end evidence (GPU box): default bench line, then rocprofv3 --kernel-trace --stats of the
# same bench command (cpu leg skipped under the profiler), summarised per kernel and launch shape.
set -o pipefail
R=$PWD; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
cd /tmp || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/rprof -o run --output-format csv -- \
  python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/bench_prof.json 2> $R/gpurun_out/bench_prof.err || exit 1
cd $R && python3 tools/ktrace_grid.py gpurun_out/rprof/run_kernel_trace.csv 40 > gpurun_out/rprof_by_grid.txt
