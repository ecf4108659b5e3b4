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
  $HIPCC $BASE "$@" -c -o build/variants/$name.k.o csrc/dcte_kernels.hip
  $HIPCC $BASE "$@" -c -o build/variants/$name.c.o csrc/dcte_capi.cpp
  $HIPCC $BASE "$@" -c -o build/variants/$name.n.o csrc/dcte_norm.hip
  $HIPCC --offload-arch=gfx950 -shared -o build/variants/$name.so build/variants/$name.k.o build/variants/$name.n.o build/variants/$name.c.o
  rm -f build/variants/$name.k.o build/variants/$name.c.o build/variants/$name.n.o
  echo built $name
}
while read -r name flags; do
  [ -z "$name" ] && continue
  build $name $flags &
done <<< "$1"
wait
