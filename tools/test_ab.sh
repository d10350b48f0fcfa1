#!/bin/bash
# GPU parity tests on the in-tree library, then the per-kernel A/B (tools/kprof_ab.sh) of the named
# variants against it; stops at the first failure.   tools/test_ab.sh tag variant ...
set -o pipefail
R=$PWD; TAG=$1; shift; O=$R/gpurun_out/$TAG; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
bash tools/kprof_ab.sh main "$@" > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
grep -E "==|total|attn_item2_kernel<false> +1069056|mlp_rows|feat_rows_kernel<3> +294144|rowgemm_qkv2_kernel +350208" $O/ab.txt
