#!/bin/bash
# isolated attention timing (tools/attn_time.py) of the in-tree library (item2 / pipe) and $VAR_DIR variants
# (all with MMPFN_ATTN_PIPE=1) at config E and C, two rounds:  tools/pipe_ab2.sh variant ...
set -o pipefail
D=${VAR_DIR:-abvar}
for round in 1 2; do
  for v in item2 pipe "$@"; do
    lib=$PWD/multimodalpfn_amd/libmmpfn_hip.so; pp=1
    [ $v = item2 ] && pp=0
    [ $v != item2 ] && [ $v != pipe ] && lib=$PWD/$D/libmmpfn_var_$v.so
    for shape in E C; do
      if [ $shape = E ]; then env="ATT_T=11 ATT_S=12000 ATT_N=10000"; reps=10; else env="ATT_T=72"; reps=40; fi
      echo -n "$shape $v r$round: "
      env $env MMPFN_DIAGNOSTICS=1 MMPFN_LIB=$lib MMPFN_ATTN_PIPE=$pp timeout -k 10 120 python3 tools/attn_time.py $reps 2>&1 | grep -v amdgpu.ids || exit 1
    done
  done
done
