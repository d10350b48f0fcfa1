#!/bin/bash
# DESIGN.md section-5 table source: kernel trace of two-member batched bf16 forwards run one at
# a time (no lane overlap), per kernel and launch shape
set -o pipefail
R=$PWD; mkdir -p gpurun_out; export TMPDIR=/tmp
cd /tmp || exit 1
MMPFN_PROF_BATCH=2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ltab -o run --output-format csv -- \
  python3 $R/tools/prof_forward.py 2 > $R/gpurun_out/ltab.log 2>&1 || exit 1
cd $R && python3 tools/ktrace_grid.py gpurun_out/ltab/run_kernel_trace.csv 30 > gpurun_out/layer_table.txt
