#!/bin/bash
# Build attention variants (local, CPU): tools/attn_variants.sh build "name:-DFLAGS" ...
# Time them (GPU box):                  tools/attn_variants.sh run name ...
set -o pipefail
C=multimodalpfn_amd/csrc
if [ "$1" = build ]; then
  shift
  for spec in "$@"; do
    name=${spec%%:*}; flags=${spec#*:}
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -mllvm -amdgpu-mfma-vgpr-form=1 -fno-honor-nans \
      $flags -x hip -c $C/attention.hip -o /tmp/attn_$name.o || exit 1
    objs=$(ls $C/build/*.o | grep -v attention)
    /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o multimodalpfn_amd/libmmpfn_var_$name.so $objs /tmp/attn_$name.o || exit 1
    echo built $name
  done
else
  shift
  mkdir -p gpurun_out
  for name in "$@"; do
    MMPFN_DIAGNOSTICS=1 MMPFN_LIB=multimodalpfn_amd/libmmpfn_var_$name.so timeout -k 10 120 python3 tools/attn_time.py 50 || exit 1
  done
fi
