#!/bin/bash
# GPU: headline step A/B between library variants (short bench, no side legs), interleaved twice
#   tools/bench_ab.sh name ...   ("main" = the in-tree library)
set -o pipefail
for round in 1 2; do for v in "$@"; do
  lib=$PWD/${VAR_DIR:-multimodalpfn_amd}/libmmpfn_var_$v.so; [ $v = main ] && lib=$PWD/multimodalpfn_amd/libmmpfn_hip.so
  echo -n "$v r$round: "
  MMPFN_DIAGNOSTICS=1 MMPFN_LIB=$lib timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-modality --no-f32 \
    --no-config-d --api-steps 0 --no-kv-cache --attn-reps 3 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" || exit 1
done; done
