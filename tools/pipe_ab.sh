#!/bin/bash
# A/B of the sample-axis attention kernels on one box (isolated launches, tools/attn_time.py):
# attn_item2 (MMPFN_ATTN_PIPE=0) vs attn_pipe (=1) at config C (T = 72: a batched pair) and E,
# two interleaved rounds, then the item-attention parity tests on the pipelined kernel.
set -o pipefail
mkdir -p gpurun_out
for round in 1 2; do for v in 0 1; do
  echo -n "C pipe=$v r$round: "; MMPFN_ATTN_PIPE=$v ATT_T=72 timeout -k 10 120 python3 tools/attn_time.py 40 || exit 1
  echo -n "E pipe=$v r$round: "; MMPFN_ATTN_PIPE=$v ATT_T=11 ATT_S=12000 ATT_N=10000 timeout -k 10 120 python3 tools/attn_time.py 10 || exit 1
done; done
[ -n "$NO_TESTS" ] && exit 0
MMPFN_ATTN_PIPE=1 timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py -k "item_attention" -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pipe_tests.log 2>&1
rc=$?; tail -5 gpurun_out/pipe_tests.log; exit $rc
