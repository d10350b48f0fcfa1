#!/bin/bash
# Isolated attention-layer timing (tools/attn_time.py) of variant libraries in $VAR_DIR (default abvar),
# config C (T = 72 columns: a batched pair) and E (T = 11, 10k keys), 2 interleaved rounds:
#   tools/attn_ab3.sh name ...   ($VAR_DIR/libmmpfn_var_<name>.so; "prod" = the in-tree library)
set -o pipefail
D=${VAR_DIR:-abvar}
for round in 1 2; do for v in "$@"; do
  lib=$PWD/$D/libmmpfn_var_$v.so; [ $v = prod ] && lib=$PWD/multimodalpfn_amd/libmmpfn_hip.so
  echo -n "C $v r$round: "; MMPFN_DIAGNOSTICS=1 MMPFN_LIB=$lib ATT_T=72 timeout -k 10 120 python3 tools/attn_time.py 40 || exit 1
  echo -n "E $v r$round: "; MMPFN_DIAGNOSTICS=1 MMPFN_LIB=$lib ATT_T=11 ATT_S=12000 ATT_N=10000 timeout -k 10 120 python3 tools/attn_time.py 10 || exit 1
done; done
