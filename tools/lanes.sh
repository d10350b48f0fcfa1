set -o pipefail
K="lanes or engine_deterministic or batch or bf16" bash tools/iter.sh || exit 1
for LB in "1 1" "2 1" "1 2" "2 2" "1 4"; do set -- $LB; timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --api-steps 0 --lanes $1 --batch $2 > gpurun_out/lb_$1_$2.json 2>gpurun_out/lb_$1_$2.err || exit 1; python3 -c "import json;d=json.load(open('gpurun_out/lb_$1_$2.json'));print('lanes $1 batch $2', d['value'], d['ms_per_step'])"; done
