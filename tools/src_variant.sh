#!/bin/bash
# Diagnostics-only variant (local, CPU): a copy of csrc/ with a sed script applied to one source, built
# into $VAR_DIR/libmmpfn_var_<name>.so with the variant marker (never the product library):
#   tools/src_variant.sh name file.hip 'sed-script' [extra hipcc flags]
set -o pipefail
name=$1; file=$2; script=$3; flags=$4
D=${VAR_DIR:-abvar}; mkdir -p $D
T=/tmp/src_var_$name; rm -rf $T; mkdir -p $T/m/csrc $T/obj $T/include
# same relative layout as the repo (sources include ../../include/*.h)
cp multimodalpfn_amd/csrc/*.hip multimodalpfn_amd/csrc/*.cpp multimodalpfn_amd/csrc/*.h multimodalpfn_amd/csrc/Makefile $T/m/csrc/
cp include/*.h $T/include/
sed -i -e "$script" $T/m/csrc/$file || exit 1
cmp -s $T/m/csrc/$file multimodalpfn_amd/csrc/$file && { echo "sed changed nothing"; exit 1; }
srcs=$(sed -n '/^SRCS :=/,/^OBJS/p' $T/m/csrc/Makefile | grep -v '^OBJS' | sed 's/SRCS :=//; s/\\//g')
for src in $srcs; do
  extra=""; { [ $src = attention.hip ] || [ $src = attention_pipe.hip ] || [ $src = featrow.hip ]; } && extra="-fno-honor-nans"
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -mllvm -amdgpu-mfma-vgpr-form=1 \
    $extra $flags -x hip -c $T/m/csrc/$src -o $T/obj/$src.o || touch $T/FAILED &
done
wait
[ -e $T/FAILED ] && { echo "compile failed"; exit 1; }
printf 'const char *const mmpfn_variant_flags = "%s";\n' "$name: $file" > $T/obj/variant_marker.c
gcc -fPIC -c $T/obj/variant_marker.c -o $T/obj/variant_marker.o || exit 1
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $D/libmmpfn_var_$name.so $T/obj/*.o && echo built $D/libmmpfn_var_$name.so
