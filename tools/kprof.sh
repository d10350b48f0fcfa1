#!/bin/bash
# rocprofv3 kernel stats of a short bench (lanes 1, so per-kernel durations do not overlap)
set -o pipefail
R=$PWD; mkdir -p gpurun_out; export TMPDIR=/tmp; cd /tmp || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/kprof -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --api-steps 0 --lanes 1 --batch 1 --attn-reps 5 > $R/gpurun_out/kprof.json 2> $R/gpurun_out/kprof.err || exit 1
cd $R && python3 tools/kstats.py gpurun_out/kprof/run_kernel_stats.csv 14
