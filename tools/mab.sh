bash tools/variants.sh prof mbase mnostore mbase mnostore > gpurun_out/mab.txt 2>&1
