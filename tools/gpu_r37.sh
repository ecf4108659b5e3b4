#!/bin/bash
# N = 4 second pass in scaled form: GPU tests, then an interleaved A/B
# against the previous commit at 16384^2 N = 4.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest exit $rc" >> "$OUT/pytest_gpu.log"; tail -4 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
V=dct-carver_amd/build/variants
: > "$OUT/ab_r37.jsonl"
timeout -k 10 300 python tools/kbench.py --n 4 --rounds 15 $V/prev.so $V/base.so >> "$OUT/ab_r37.jsonl" || exit 1
timeout -k 10 300 python tools/kbench.py --n 4 --rounds 15 $V/prev.so $V/base.so >> "$OUT/ab_r37.jsonl" || exit 1
cat "$OUT/ab_r37.jsonl"
