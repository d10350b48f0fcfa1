#!/bin/bash
# PMC passes (separate rocprofv3 runs, --pmc only with kernel stats; no trace domains).
# Writes gpurun_out/pmc_<name>/ csv files.  Each step time-bounded; stops at the first failure.
set -o pipefail
R=$PWD
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 120 rocprofv3 -L > $R/gpurun_out/pmc_list.txt 2>&1 || true
run() {  # name counters...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" -d $R/gpurun_out/pmc_$name -o run --output-format csv -- \
    python3 $R/tools/prof_forward.py 2 > $R/gpurun_out/pmc_$name.log 2>&1
}
run fetch FETCH_SIZE &&
run write WRITE_SIZE &&
run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS &&
run sq2 SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM &&
run sq3 SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT
echo "pmc_rc=$?"
