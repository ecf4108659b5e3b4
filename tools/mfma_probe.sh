#!/bin/bash
# Build (if needed) and run tools/mfma_probe.hip: MFMA 4x4x1 layout, fmaf-chain
# numerics and VALU/MFMA co-issue costs on the box's GPU.
set -e
cd "$(dirname "$0")"
[ -x bin/mfma_probe ] || { mkdir -p bin; hipcc -O3 -Wno-unused-value --offload-arch=gfx950 -o bin/mfma_probe mfma_probe.hip; }
timeout -k 10 60 bin/mfma_probe
