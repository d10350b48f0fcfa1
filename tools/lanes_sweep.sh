#!/bin/bash
# Headline step at several (lanes, members per batched forward) settings, headline pass only.
set -o pipefail
R=$PWD; O=$R/gpurun_out/lanes; mkdir -p $O
for lb in "2 2" "1 4" "2 1" "4 1" "1 2" "3 1"; do
  set -- $lb
  timeout -k 10 200 python bench.py --lanes $1 --batch $2 --steps 20 --warmup 5 --no-cpu-baseline --no-modality \
    --no-f32 --no-config-d --no-kv-cache --api-steps 0 --attn-reps 2 > $O/l$1b$2.json 2> $O/l$1b$2.err || exit 1
  python3 -c "import json;d=json.load(open('$O/l$1b$2.json'));print('lanes $1 batch $2', d['value'], d['ms_per_step'])"
done
