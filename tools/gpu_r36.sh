#!/bin/bash
# N = 16 edge columns (k1 = 0, 1) in the scaled forms too: GPU tests, then an
# interleaved A/B against the previous commit at 8192^2 N = 16, with the
# N = 16 VGPR cap at 4 / 3 / 2 waves per SIMD.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest exit $rc" >> "$OUT/pytest_gpu.log"; tail -4 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
V=dct-carver_amd/build/variants
: > "$OUT/ab_r36.jsonl"
timeout -k 10 300 python tools/kbench.py --n 16 --size 8192 --rounds 15 $V/prev.so $V/base.so $V/mw3.so $V/mw2.so >> "$OUT/ab_r36.jsonl" || exit 1
timeout -k 10 300 python tools/kbench.py --n 16 --size 8192 --rounds 15 $V/prev.so $V/base.so $V/mw3.so $V/mw2.so >> "$OUT/ab_r36.jsonl" || exit 1
cat "$OUT/ab_r36.jsonl"
