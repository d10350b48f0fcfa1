#!/bin/bash
# GPU: rocprofv3 kernel stats of tools/prof_forward.py (two-member batched forwards, one lane) for
# each library variant; prints the per-kernel average durations side by side.
#   tools/kvar.sh name ...   (multimodalpfn_amd/libmmpfn_var_<name>.so; "main" = the in-tree library)
set -o pipefail
R=$PWD; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in "$@"; do
  lib=$R/multimodalpfn_amd/libmmpfn_var_$v.so; [ $v = main ] && lib=$R/multimodalpfn_amd/libmmpfn_hip.so
  (cd /tmp && MMPFN_DIAGNOSTICS=1 MMPFN_LIB=$lib MMPFN_PROF_BATCH=2 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/kvar_$v -o run \
     --output-format csv -- python3 $R/tools/prof_forward.py 4 > $R/gpurun_out/kvar_$v.log 2>&1) || exit 1
  echo "== $v"; python3 tools/kstats.py gpurun_out/kvar_$v/run_kernel_stats.csv 8
done
