#!/bin/bash
# PMC passes (FETCH_SIZE; TCC_HIT/MISS; TCC_EA0_RDREQ) over one forward, rows of the MGM GLU GEMM kernel
set -o pipefail
R=$PWD; mkdir -p gpurun_out; export TMPDIR=/tmp
cd /tmp || exit 1
i=0
for c in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $c -d $R/gpurun_out/gpmc_$i -o run --output-format csv -- \
    python3 $R/tools/prof_forward.py 1 > $R/gpurun_out/gpmc_$i.log 2>&1 || exit 1
done
cd $R && for i in 1 2 3; do grep -h "glu_big\|gemm_kernel<true, false, false, 4>" gpurun_out/gpmc_$i/run_counter_collection.csv | awk -F, '{print $(NF-1), $NF}' | sort | uniq -c | head; done
