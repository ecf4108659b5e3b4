#!/bin/bash
# A/B: wave priority while staging / converting, single-buffered path (N = 16, 8192^2)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
V=dct-carver_amd/build/variants
timeout -k 10 300 python tools/kbench.py --n 16 --size 8192 --rounds 9 $V/p16a.so $V/p16b.so > "$OUT/ab_r25.jsonl" 2> "$OUT/ab_r25.err" || { echo "ab failed"; tail -5 "$OUT/ab_r25.err"; exit 1; }
cat "$OUT/ab_r25.jsonl"
