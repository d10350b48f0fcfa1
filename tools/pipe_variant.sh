#!/bin/bash
# Diagnostics-only variants of attention_pipe.hip (local, CPU): a sed script applied to a temporary copy,
# linked with the in-tree objects into $VAR_DIR/libmmpfn_var_<name>.so (never the product library):
#   tools/pipe_variant.sh name 'sed-script' [extra hipcc flags]
set -o pipefail
name=$1; script=$2; flags=$3
D=${VAR_DIR:-abvar}; mkdir -p $D
C=multimodalpfn_amd/csrc
T=/tmp/pipe_var_$name; mkdir -p $T
sed -e "$script" ${SRC:-$C/attention_pipe.hip} > $T/attention_pipe.hip || exit 1
cp $C/common.h $C/kernels.h $T/
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -mllvm -amdgpu-mfma-vgpr-form=1 \
  -fno-honor-nans $flags -x hip -c $T/attention_pipe.hip -o $T/attention_pipe.o || exit 1
printf 'const char *const mmpfn_variant_flags = "%s";\n' "pipe $name" > $T/marker.c
gcc -fPIC -c $T/marker.c -o $T/marker.o || exit 1
objs=$(ls $C/build/*.o | grep -v attention_pipe)
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $D/libmmpfn_var_$name.so $objs $T/attention_pipe.o $T/marker.o && echo built $D/libmmpfn_var_$name.so
