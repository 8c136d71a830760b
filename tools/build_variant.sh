#!/bin/bash
# A/B variant of the batched pipeline kernels (diagnostics, tools/ab.py): compiles the
# kernels_w4_t8 translation unit (the 512-wide policies' and GRU-256's instantiations; UNITS="t2 t4 t8" for more)
# with extra compiler flags / defines, links it with the default objects of every other
# unit into lib/diag/libgo2pi_<name>.so.
#   tools/build_variant.sh vgpr -mllvm -amdgpu-mfma-vgpr-form
set -e
name=$1
shift
C=$(cd "$(dirname "$0")/../go2_onnx_controller_amd/csrc" && pwd)
L=$C/../lib
mkdir -p $L/diag/$name
cd $C
# UNITS: the pipeline units built with the flags (default t8); the others are the default objects
objs=""
for t in t2 t4 t8; do
  if [[ " ${UNITS:-t8} " == *" $t "* ]]; then
    /opt/rocm/bin/hipcc -O3 -std=c++20 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -I../../include \
      -mllvm -amdgpu-kernarg-preload-count=16 "$@" -c kernels_w4_$t.hip -o $L/diag/$name/kernels_w4_$t.o &
    objs="$objs $L/diag/$name/kernels_w4_$t.o"
  else
    objs="$objs $L/kernels_w4_$t.o"
  fi
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $L/diag/libgo2pi_$name.so $L/kernels.o $objs \
  $L/kernels_gen_w4.o $L/kernels_gen_w8.o $L/kernels_gen_w16.o $L/resident.o $L/resident_wide.o $L/engine.o \
  $L/onnx_model.o
echo "built $L/diag/libgo2pi_$name.so"
