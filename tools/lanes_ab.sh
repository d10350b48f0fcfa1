#!/bin/bash
# Alternating A/B of two (lanes, batch) settings of the headline step: tools/lanes_ab.sh "2 2" "2 1" [rounds]
set -o pipefail
R=$PWD; O=$R/gpurun_out/lanes_ab; mkdir -p $O
A=$1; B=$2; N=${3:-3}
for i in $(seq 1 $N); do
  for lb in "$A" "$B"; do
    set -- $lb
    timeout -k 10 200 python bench.py --lanes $1 --batch $2 --steps 30 --warmup 5 --no-cpu-baseline --no-modality \
      --no-f32 --no-config-d --no-kv-cache --api-steps 0 --attn-reps 2 > $O/r.json 2> $O/r.err || exit 1
    python3 -c "import json;d=json.load(open('$O/r.json'));print('lanes $1 batch $2', d['value'], d['ms_per_step'])"
  done
done
