#!/bin/bash
# GPU: the e4m3 P.V attention variant (build: tools/build_variant.sh f8 -DMMPFN_ATTN_FP8PV) against
# the in-tree bf16 kernel: isolated launch time at the C (T = 72) and E shapes, and config-E logits.
set -o pipefail
for v in main f8; do
  lib=$PWD/multimodalpfn_amd/libmmpfn_var_$v.so; [ $v = main ] && lib=$PWD/multimodalpfn_amd/libmmpfn_hip.so
  for sh in "72 2298 1838" "11 12000 10000"; do set -- $sh
    echo -n "$v T=$1 S=$2: "; MMPFN_DIAGNOSTICS=1 MMPFN_LIB=$lib ATT_T=$1 ATT_S=$2 ATT_N=$3 timeout -k 10 120 python3 tools/attn_time.py 20 || exit 1
  done
  MMPFN_DIAGNOSTICS=1 MMPFN_LIB=$lib timeout -k 10 200 python3 tools/e_logits.py $v 2>&1 | grep -v amdgpu.ids || exit 1
done
