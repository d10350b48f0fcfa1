#!/bin/bash
# round 5 GPU pass: the GPU test suite, the printed parity numbers of the fp16 / fp8 tests, the 1-GPU bench and the
# launcher rehearsal (`python bench.py --gpus 2`, two gloo ranks on one GPU).  $1: output tag
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -m gpu -q -s --timeout 300 --timeout-method thread \
  -k "f16_mode_within or fp8 or f16_close" > $O/pytest_numbers.log 2>&1 || { tail -40 $O/pytest_numbers.log; exit 1; }
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
tail -n 1 $O/bench.json | head -c 400; echo
bash tools/rehearse_multirank.sh && cp -r gpurun_out/rehearse $O/
