#!/bin/bash
# GPU: attention kernel tests + isolated launch timing (C shape T = 72 and E shape) for library variants
#   tools/attn_ab2.sh name ...   ("main" = the in-tree library)
set -o pipefail
for v in "$@"; do
  lib=$PWD/multimodalpfn_amd/libmmpfn_var_$v.so; [ $v = main ] && lib=$PWD/multimodalpfn_amd/libmmpfn_hip.so
  MMPFN_DIAGNOSTICS=1 MMPFN_LIB=$lib timeout -k 10 200 python3 -m pytest tests/test_parity_gpu.py -q -x -k "item_attention" --timeout 120 \
    --timeout-method thread -p no:cacheprovider 2>&1 | tail -1 || exit 1
done
for round in 1 2; do for v in "$@"; do
  lib=$PWD/multimodalpfn_amd/libmmpfn_var_$v.so; [ $v = main ] && lib=$PWD/multimodalpfn_amd/libmmpfn_hip.so
  for sh in "72:2298:1838" "11:12000:10000"; do IFS=: read t sr nr <<< "$sh"
    echo -n "$v r$round T=$t: "; MMPFN_DIAGNOSTICS=1 MMPFN_LIB=$lib ATT_T=$t ATT_S=$sr ATT_N=$nr timeout -k 10 120 python3 tools/attn_time.py 30 || exit 1
  done
done; done
