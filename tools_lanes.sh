set -o pipefail
K="lanes or engine_deterministic" bash tools_iter.sh || exit 1
for L in 1 2 4; do timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --api-steps 0 --lanes $L > gpurun_out/lanes_$L.json 2>gpurun_out/lanes_$L.err || exit 1; python3 -c "import json;d=json.load(open('gpurun_out/lanes_$L.json'));print($L, d['value'], d['ms_per_step'])"; done
