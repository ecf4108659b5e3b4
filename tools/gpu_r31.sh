#!/bin/bash
# Scaled k0 column too (dct8_k0_sc): GPU tests on the default build, then an
# interleaved A/B against the previous kernel (SC=0, 256 threads).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest exit $rc" >> "$OUT/pytest_gpu.log"; tail -15 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
V=dct-carver_amd/build/variants
L="$V/old.so $V/new.so $V/new64.so"
: > "$OUT/ab_r31.jsonl"
timeout -k 10 300 python tools/kbench.py --n 8 --rounds 15 $L >> "$OUT/ab_r31.jsonl" || exit 1
timeout -k 10 300 python tools/kbench.py --n 8 --rounds 15 $L >> "$OUT/ab_r31.jsonl" || exit 1
cat "$OUT/ab_r31.jsonl"
