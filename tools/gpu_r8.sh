#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
rc=$?
echo "pytest exit $rc" >> "$OUT/pytest_gpu.log"; tail -15 "$OUT/pytest_gpu.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/kbench.py --n 8 dct-carver_amd/build/libdctenergy_hip.so > "$OUT/ab8.jsonl" 2>"$OUT/ab8.err" || { tail -5 "$OUT/ab8.err"; exit 1; }
cat "$OUT/ab8.jsonl"
