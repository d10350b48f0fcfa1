#!/bin/bash
# SQ / GRBM counters of the sample-axis attention kernel alone (tools/attn_time.py at ATT_T
# token columns), one rocprofv3 --pmc pass per counter set, each time-bounded:
#   tools/attn_sq_pmc.sh [lib.so]   -> gpurun_out/attn_sq/<pass>/run_counter_collection.csv
set -o pipefail
export ATT_T=${ATT_T:-72}
R=$PWD; O=${OUT:-attn_sq}; mkdir -p gpurun_out/$O; export TMPDIR=/tmp
LIB=${1:-}
cd /tmp || exit 1
pass() {
  local name=$1; shift
  MMPFN_DIAGNOSTICS=1 MMPFN_LIB=$LIB timeout -s KILL 90 rocprofv3 --pmc "$@" -d $R/gpurun_out/$O/$name -o run --output-format csv -- \
    python3 $R/tools/attn_time.py ${REPS:-5} > $R/gpurun_out/$O/$name.log 2>&1
}
pass a SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT || exit 1
pass b ${PASS_B:-SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_TRANS_F32 SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS} || exit 1
cd $R && python3 tools/attn_sq_summary.py gpurun_out/$O > gpurun_out/$O/summary.txt && cat gpurun_out/$O/summary.txt
