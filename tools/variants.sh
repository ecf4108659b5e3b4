#!/bin/bash
# Build libdctenergy_hip.so variants (tuning knobs as -D flags) into
# dct-carver_amd/build/variants/<name>.so; run on the box with tools/kbench.py.
set -e
cd "$(dirname "$0")/../dct-carver_amd"
mkdir -p build/variants
HIPCC=/opt/rocm/bin/hipcc
BASE="-O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize -fPIC --offload-arch=gfx950"
build() {  # name extra-flags...
  local name=$1; shift
  local objs=""
  for src in csrc/dcte_kernels.hip csrc/dcte_exact.hip csrc/dcte_norm.hip csrc/dcte_seam.hip csrc/dcte_dp.hip csrc/dcte_capi.cpp; do
    local o=build/variants/$name.$(basename $src).o
    $HIPCC $BASE "$@" -c -o $o $src
    objs="$objs $o"
  done
  local ho=build/variants/$name.dcte_host.o
  g++ -O3 -std=c++17 -ffp-contract=off -fPIC -c -o $ho csrc/dcte_host.cpp
  objs="$objs $ho"
  $HIPCC --offload-arch=gfx950 -shared -o build/variants/$name.so $objs
  rm -f $objs
  echo built $name
}
while read -r name flags; do
  [ -z "$name" ] && continue
  build $name $flags &
done <<< "$1"
wait
