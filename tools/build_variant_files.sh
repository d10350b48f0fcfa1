#!/bin/bash
# Variant library with extra flags on SOME sources only (the rest from the in-tree build/ objects):
#   tools/build_variant_files.sh name "flags" file.hip [file.hip ...]
set -o pipefail
mkdir -p ${VAR_DIR:-multimodalpfn_amd}
name=$1; flags=$2; shift 2
C=multimodalpfn_amd/csrc; B=/tmp/mmpfn_varf_$name
make -C $C -s >/dev/null || exit 1
rm -rf $B; mkdir -p $B; cp $C/build/*.o $B/
for src in "$@"; do
  extra=""; { [ $src = attention.hip ] || [ $src = featrow.hip ]; } && extra="-fno-honor-nans"
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -mllvm -amdgpu-mfma-vgpr-form=1 \
    $extra $flags -x hip -c $C/$src -o $B/$src.o || exit 1
done
printf 'const char *const mmpfn_variant_flags = "%s";\n' "$name: $flags" > $B/variant_marker.c
gcc -fPIC -c $B/variant_marker.c -o $B/variant_marker.o || exit 1
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ${VAR_DIR:-multimodalpfn_amd}/libmmpfn_var_$name.so $B/*.o && echo built $name
