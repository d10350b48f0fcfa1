#!/bin/bash
# Two SQ counter passes (<= 8 SQ counters each) over batched bf16 forwards (MMPFN_PROF_BATCH=2, the
# bench's launch shape) and a per-kernel summary of where each layer kernel's wave cycles go.
set -o pipefail
R=$PWD; TAG=${1:-lpmc}; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp MMPFN_PROF_BATCH=2
cd /tmp || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
  SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_MFMA -d $O/a -o run --output-format csv -- \
  python3 $R/tools/prof_forward.py 1 > $O/a.log 2>&1 || { tail -5 $O/a.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
  SQ_ACTIVE_INST_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE -d $O/b -o run --output-format csv -- \
  python3 $R/tools/prof_forward.py 1 > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
cd $R && python3 tools/layer_pmc_summary.py $O/a/run_counter_collection.csv $O/b/run_counter_collection.csv | tee $O/summary.txt
