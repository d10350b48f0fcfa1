#!/bin/bash
# HBM traffic of the headline kernel (attn_pipe_kernel) at the bench shape: two separate
# rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; no trace domains) over tools/attn_time.py,
# summarised (gfx950 FETCH_SIZE x2 correction) into gpurun_out/attn_pipe_pmc_T$ATT_T.json
# (ATT_T = token columns per launch: 36 one member, 72 the bench's two-member batched forward).
set -o pipefail
export ATT_T=${ATT_T:-36}
R=$PWD
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 120 rocprofv3 --pmc $c -d $R/gpurun_out/apmc_$c -o run --output-format csv -- \
    python3 $R/tools/attn_time.py 5 > $R/gpurun_out/apmc_$c.log 2>&1 || exit 1
done
cd $R && python3 tools/attn_pmc_summary.py gpurun_out/apmc_FETCH_SIZE gpurun_out/apmc_WRITE_SIZE > gpurun_out/attn_pipe_pmc_T$ATT_T${ATT_PREC:+_$ATT_PREC}.json
