#!/bin/bash
# Decision by selects instead of fmaxf/fminf (no canonicalising ops):
# GPU tests, then interleaved A/Bs against the previous commit
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest exit $rc" >> "$OUT/pytest_gpu.log"; tail -4 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
V=dct-carver_amd/build/variants
: > "$OUT/ab_r41.jsonl"
timeout -k 10 300 python tools/kbench.py --n 8 --rounds 15 $V/prev.so $V/base.so >> "$OUT/ab_r41.jsonl" || exit 1
timeout -k 10 300 python tools/kbench.py --n 16 --size 8192 --rounds 15 $V/prev.so $V/base.so >> "$OUT/ab_r41.jsonl" || exit 1
timeout -k 10 300 python tools/kbench.py --n 8 --rounds 15 $V/prev.so $V/base.so >> "$OUT/ab_r41.jsonl" || exit 1
cat "$OUT/ab_r41.jsonl"
