#!/bin/bash
# bench value per (lanes, batch) combination, 2 interleaved rounds (GPU box)
set -o pipefail
mkdir -p gpurun_out
for round in 1 2; do
  for lb in "2 2" "4 1" "1 4" "2 1"; do
    set -- $lb
    timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --api-steps 0 --attn-reps 5 \
      --no-kv-cache --lanes $1 --batch $2 > gpurun_out/lab.json 2> gpurun_out/lab.err || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/lab.json')); print('lanes $1 batch $2', d['value'], d['ms_per_step'])"
  done
done
