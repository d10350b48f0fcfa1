#!/bin/bash
# GPU: the new config / seam tests (bounded), parity log kept under gpurun_out/
set -o pipefail
mkdir -p gpurun_out
export MMPFN_PARITY_LOG=$PWD/gpurun_out/parity_bf16.jsonl
rm -f $MMPFN_PARITY_LOG
timeout -k 10 900 python -u -m pytest tests/test_configs_gpu.py -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_new.log 2>&1
rc=$?; echo "pytest_rc=$rc" >> gpurun_out/pytest_new.log; tail -25 gpurun_out/pytest_new.log; exit $rc
