#!/bin/bash
# Config B forwards in a kernel trace: a short bench with the config-B leg (rocprofv3 --kernel-trace --stats; two lanes,
# so kernel times overlap).  $1: output tag
set -o pipefail
R=$PWD; O=$R/gpurun_out/${1:-configb}; mkdir -p $O; export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/rprof -o run --output-format csv -- \
  python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-modality --no-f32 --no-config-d --no-config-e \
  --api-steps 0 --no-kv-cache --attn-reps 2 > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
cd $R && python3 tools/ktrace_grid.py $O/rprof/run_kernel_trace.csv 40 > $O/by_grid.txt && head -40 $O/by_grid.txt
