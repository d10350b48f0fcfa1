#!/bin/bash
# GPU: kernel stats of one ViT-B/14 bf16 forward batch per library variant (tools/variants.sh build, SRC=modality)
#   tools/mod_var.sh name ...   (name "main" = the in-tree library)
set -o pipefail
R=$PWD; mkdir -p gpurun_out; export TMPDIR=/tmp ITERS=2
for name in "$@"; do
  lib=$R/multimodalpfn_amd/libmmpfn_var_$name.so; [ "$name" = main ] && lib=$R/multimodalpfn_amd/libmmpfn_hip.so
  cd /tmp && MMPFN_DIAGNOSTICS=1 MMPFN_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/mvar_$name -o run \
    --output-format csv -- python3 $R/tools/modality_prof.py vit bf16 128 > $R/gpurun_out/mvar_$name.log 2>&1 || exit 1
  cd $R && echo "== $name" && python3 tools/kstats.py gpurun_out/mvar_$name/run_kernel_stats.csv 5
done
