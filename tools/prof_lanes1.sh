#!/bin/bash
# rocprofv3 kernel trace + stats of the headline step at one lane (kernels one after another): the
# per-kernel durations the bench line's `roofline` (one-lane pass) is measured on.
set -o pipefail
R=$PWD; TAG=${1:-run}; O=$R/gpurun_out/${TAG}_lanes1; mkdir -p $O; export TMPDIR=/tmp  # own dir: evidence.sh writes $TAG
cd /tmp || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/rprof -o run --output-format csv -- \
  python3 $R/bench.py --precision ${PREC:-f16} --lanes 1 --steps 10 --warmup 3 --no-cpu-baseline --no-modality --no-config-d --no-config-e --no-config-b --no-f32 \
  --api-steps 0 --no-kv-cache --attn-reps 5 > $O/bench_l1.json 2> $O/bench_l1.err || { tail -5 $O/bench_l1.err; exit 1; }
cd $R && python3 tools/ktrace_grid.py $O/rprof/run_kernel_trace.csv 30 > $O/rprof_by_grid.txt && head -24 $O/rprof_by_grid.txt
