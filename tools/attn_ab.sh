#!/bin/bash
# isolated attention-layer timing (tools/attn_time.py) of library variants, 2 interleaved rounds:
#   tools/attn_ab.sh name ...   (multimodalpfn_amd/libmmpfn_var_<name>.so)
set -o pipefail
mkdir -p gpurun_out
for round in 1 2; do for v in "$@"; do
  echo -n "$v r$round: "; MMPFN_DIAGNOSTICS=1 MMPFN_LIB=$PWD/multimodalpfn_amd/libmmpfn_var_$v.so timeout -k 10 120 python3 tools/attn_time.py 100 || exit 1
done; done
