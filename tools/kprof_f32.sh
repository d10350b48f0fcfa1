#!/bin/bash
# rocprofv3 kernel stats of the parity-mode step (bench.py --precision f32, lanes 1, 2 steps)
set -o pipefail
R=$PWD; mkdir -p gpurun_out; export TMPDIR=/tmp; cd /tmp || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/kprof_f32 -o run --output-format csv -- python3 $R/bench.py --precision f32 --steps 2 --warmup 1 --no-cpu-baseline --api-steps 0 --lanes 1 --attn-reps 2 --no-kv-cache --no-config-d --no-modality --no-f32 > $R/gpurun_out/kprof_f32.json 2> $R/gpurun_out/kprof_f32.err || exit 1
cd $R && python3 tools/kstats.py gpurun_out/kprof_f32/run_kernel_stats.csv 16
