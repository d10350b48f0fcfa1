#!/bin/bash
# rocprofv3 kernel trace of a short bench (lanes 1 x batch 2: the bench's launch shapes, no overlap) per
# library variant, summarised per (kernel, grid):   tools/kprof_ab.sh name ...   ("main" = in-tree)
set -o pipefail
R=$PWD; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in "$@"; do
  lib=$R/${VAR_DIR:-multimodalpfn_amd}/libmmpfn_var_$v.so; [ $v = main ] && lib=$R/multimodalpfn_amd/libmmpfn_hip.so
  cd /tmp || exit 1
  MMPFN_DIAGNOSTICS=1 MMPFN_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/kp_$v -o run --output-format csv -- \
    python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-modality --no-f32 --no-config-d --api-steps 0 \
    --no-kv-cache --no-config-e --no-config-b --lanes 1 --batch 2 --attn-reps 2 > $R/gpurun_out/kp_$v.json 2> $R/gpurun_out/kp_$v.err || exit 1
  cd $R && echo "== $v" && python3 tools/ktrace_grid.py gpurun_out/kp_$v/run_kernel_trace.csv 12 || exit 1
done
