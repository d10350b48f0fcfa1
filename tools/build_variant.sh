#!/bin/bash
# Build the whole engine with extra compile flags into multimodalpfn_amd/libmmpfn_var_<name>.so
# (local, CPU):  tools/build_variant.sh name "-DFLAG=1 ..."
set -o pipefail
mkdir -p ${VAR_DIR:-multimodalpfn_amd}
name=$1; flags=$2
C=multimodalpfn_amd/csrc
B=/tmp/mmpfn_var_$name
mkdir -p $B
srcs=$(sed -n '/^SRCS :=/,/^OBJS/p' $C/Makefile | grep -v '^OBJS' | sed 's/SRCS :=//; s/\\//g')
for src in $srcs; do
  extra=""; { [ $src = attention.hip ] || [ $src = attention_pipe.hip ] || [ $src = featrow.hip ]; } && extra="-fno-honor-nans"
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -mllvm -amdgpu-mfma-vgpr-form=1 \
    $extra $flags -x hip -c $C/$src -o $B/$src.o &
done
wait
printf 'const char *const mmpfn_variant_flags = "%s";\n' "$name: $flags" > $B/variant_marker.c
gcc -fPIC -c $B/variant_marker.c -o $B/variant_marker.o || exit 1
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ${VAR_DIR:-multimodalpfn_amd}/libmmpfn_var_$name.so $B/*.o && echo built $name
