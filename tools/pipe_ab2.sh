#!/bin/bash
# isolated attention timing (tools/attn_time.py) of the in-tree library and $VAR_DIR variants
# (tools/pipe_variant.sh) at config E and C, two interleaved rounds:  tools/pipe_ab2.sh variant ...
set -o pipefail
D=${VAR_DIR:-abvar}
for round in 1 2; do
  for v in prod "$@"; do
    lib=$PWD/multimodalpfn_amd/libmmpfn_hip.so
    [ $v != prod ] && lib=$PWD/$D/libmmpfn_var_$v.so
    for shape in E C; do
      if [ $shape = E ]; then env="ATT_T=11 ATT_S=12000 ATT_N=10000"; reps=10; else env="ATT_T=72"; reps=40; fi
      echo -n "$shape $v r$round: "
      env $env MMPFN_DIAGNOSTICS=1 MMPFN_LIB=$lib timeout -k 10 120 python3 tools/attn_time.py $reps 2>&1 | grep -v amdgpu.ids || exit 1
    done
  done
done
