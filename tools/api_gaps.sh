#!/bin/bash
# kernel trace of 13 predict_proba calls at config C and the per-predict idle analysis; $1: output tag
set -o pipefail
R=$PWD; O=$R/gpurun_out/$1; mkdir -p $O; export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/apitrace -o run -- python3 $R/tools/api_gaps.py \
  > $O/api_gaps_run.log 2>&1 || { tail -20 $O/api_gaps_run.log; exit 1; }
cd $R && grep "ms per predict" $O/api_gaps_run.log && python3 tools/api_gaps.py --trace $O/apitrace/run_kernel_trace.csv \
  > $O/api_gaps.txt && cat $O/api_gaps.txt
