#!/bin/bash
# Kernel A/B variants.
#   build (CPU):  SRC=featrow tools/variants.sh build "name:-DFLAGS" ...   -> multimodalpfn_amd/libmmpfn_var_<name>.so
#   prof (GPU):   tools/variants.sh prof name ...   kernel stats of a 2-member bf16 forward per variant
set -o pipefail
C=multimodalpfn_amd/csrc
if [ "$1" = build ]; then
  shift
  for spec in "$@"; do
    name=${spec%%:*}; flags=${spec#*:}
    extra=""; [ "$SRC" = attention ] && extra="-fno-honor-nans"
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 ${FORM--mllvm -amdgpu-mfma-vgpr-form=1} $extra \
      $flags -x hip -c $C/$SRC.hip -o /tmp/var_$name.o || exit 1
    objs=$(ls $C/build/*.o | grep -v "/$SRC.hip.o")
    /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o multimodalpfn_amd/libmmpfn_var_$name.so $objs /tmp/var_$name.o || exit 1
    echo built $name
  done
else
  shift
  R=$PWD; mkdir -p gpurun_out; export TMPDIR=/tmp
  for name in "$@"; do
    cd /tmp && MMPFN_DIAGNOSTICS=1 MMPFN_LIB=$R/multimodalpfn_amd/libmmpfn_var_$name.so timeout -k 10 200 rocprofv3 --kernel-trace --stats \
      -d $R/gpurun_out/var_$name -o run --output-format csv -- python3 $R/tools/prof_forward.py 2 > $R/gpurun_out/var_$name.log 2>&1 || exit 1
    cd $R && echo "== $name" && python3 tools/kstats.py gpurun_out/var_$name/run_kernel_stats.csv 5
  done
fi
