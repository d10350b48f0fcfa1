#!/bin/bash
# Functional rehearsal of the multi-rank bench path on a one-GPU box (NOT a measurement): bench.py launches its
# two ranks itself (no torchrun: the form `python bench.py --gpus N` the driver may use), both on cuda:0 over gloo
# (RCCL refuses two ranks on one GPU).  The driver's N = 2/4/8 runs use RCCL, one GPU per rank.
set -o pipefail
R=$PWD; O=$R/gpurun_out/rehearse; mkdir -p $O
MMPFN_BENCH_SHARE_GPUS=1 MMPFN_BENCH_BACKEND=gloo timeout -k 10 500 python -u bench.py --gpus 2 --steps 3 --warmup 1 \
  --no-cpu-baseline --no-modality --no-f32 --no-config-b --no-config-e --no-config-b --attn-reps 2 --api-steps 1 \
  > $O/bench2.json 2> $O/bench2.err || { tail -30 $O/bench2.err; exit 1; }
tail -n 1 $O/bench2.json | head -c 1500
