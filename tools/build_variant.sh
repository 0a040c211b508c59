#!/bin/bash
# Build libvitmi.so from a modified copy of csrc/ for A/B kernel timing (load it with VITMI_LIB):
#   [VARIANT_FLAGS=-D...] tools/build_variant.sh NAME SRC_DIR   -> transformer-stm_amd/variants/NAME.so
# SRC_DIR must sit two levels below a directory holding include/ (mirror of the repo layout).
set -e
name=$1; src=$2
root=$(cd "$(dirname "$0")/.." && pwd)
out=$root/transformer-stm_amd/variants
mkdir -p $out /tmp/vb_$name
objs=""
for f in abi.cpp boundary.cpp comm.cpp gemm.hip attention.hip layernorm.hip elementwise.hip cvt.hip dense.hip optim.hip sls.hip split.hip; do
  extra=""; [ "$f" = optim.hip ] && extra=-ffp-contract=off
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $extra $VARIANT_FLAGS -c $src/$f -o /tmp/vb_$name/$f.o &
  objs="$objs /tmp/vb_$name/$f.o"
done
wait
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $out/$name.so $objs -ldl
echo built $out/$name.so
