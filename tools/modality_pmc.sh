#!/bin/bash
# PMC passes over one ViT-B/14 bf16 forward (tools/modality_prof.py, ITERS=1), one rocprofv3 --pmc
# pass per counter set, each time-bounded:  tools/modality_pmc.sh -> gpurun_out/mpmc/summary.txt
set -o pipefail
R=$PWD; mkdir -p gpurun_out/mpmc; export TMPDIR=/tmp ITERS=1
cd /tmp || exit 1
pass() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d $R/gpurun_out/mpmc/$name -o run --output-format csv -- \
    python3 $R/tools/modality_prof.py vit bf16 ${B:-128} > $R/gpurun_out/mpmc/$name.log 2>&1
}
pass a SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT || exit 1
pass b SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS || exit 1
pass c FETCH_SIZE || exit 1
pass d WRITE_SIZE || exit 1
pass e TCC_HIT_sum TCC_MISS_sum || exit 1
cd $R && python3 tools/pmc_by_kernel.py gpurun_out/mpmc/*/run_counter_collection.csv > gpurun_out/mpmc/summary.txt
