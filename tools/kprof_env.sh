#!/bin/bash
# rocprofv3 kernel trace of a short bench (lanes 1 x batch 2) per environment setting of the in-tree library,
# summarised per (kernel, grid):   tools/kprof_env.sh name=ENV=VALUE ...   ("name=" alone: no extra variable)
set -o pipefail
R=$PWD; mkdir -p gpurun_out; export TMPDIR=/tmp
for spec in "$@"; do
  name=${spec%%=*}; env_kv=${spec#*=}
  cd /tmp || exit 1
  env ${env_kv:+$env_kv} timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/ke_$name -o run --output-format csv -- \
    python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-modality --no-f32 --no-config-d --api-steps 0 \
    --no-kv-cache --no-config-e --no-config-b --lanes 1 --batch 2 --attn-reps 2 > $R/gpurun_out/ke_$name.json 2> $R/gpurun_out/ke_$name.err || exit 1
  cd $R && echo "== $name ($env_kv)" && python3 tools/ktrace_grid.py gpurun_out/ke_$name/run_kernel_trace.csv 12 || exit 1
done
