#!/bin/bash
# A/B bench of library variants in one GPU call (interleaved, 2 rounds): tools/ab_bench.sh name ...
# ("default" = the in-tree libmmpfn_hip.so).  Prints value per run.
set -o pipefail
mkdir -p gpurun_out
for round in 1 2; do
  for name in "$@"; do
    case "$name" in
      default) lib=""; envs="" ;;
      env:*) lib=""; envs="${name#env:}" ;;   # env:VAR=value  (default library)
      *) lib=multimodalpfn_amd/libmmpfn_var_$name.so; envs="" ;;
    esac
    env $envs MMPFN_DIAGNOSTICS=1 MMPFN_LIB=$lib timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --api-steps 0 \
      --attn-reps 5 > gpurun_out/ab.json 2> gpurun_out/ab.err || exit 1
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab.json')); print('$name', d['value'], d['ms_per_step'])"
  done
done
