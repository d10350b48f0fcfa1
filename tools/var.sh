# bench stability vs warmup length (diagnostic)
set -o pipefail
for cfg in "--steps 30 --warmup 5" "--steps 30 --warmup 60" "--steps 30 --warmup 150" "--steps 30 --warmup 5"; do
  timeout -k 10 300 python3 bench.py $cfg --no-cpu-baseline --api-steps 0 --no-kv-cache --attn-reps 5 > gpurun_out/v.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/v.json')); print('$cfg', d['value'], d['ms_per_step'])"
done
