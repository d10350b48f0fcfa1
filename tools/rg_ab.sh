#!/bin/bash
# isolated two-member forward kernel stats for the row-GEMM ablation variants (GPU)
set -o pipefail
bash tools/variants.sh prof rgbase rgnostore rgnostage rgnosync rgnone base prio1 prio2
