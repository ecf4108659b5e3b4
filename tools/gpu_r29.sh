#!/bin/bash
# A/B (longer): N = 8 map kernel, 256- vs 64-thread workgroups (+ G = 16, no setprio).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
V=dct-carver_amd/build/variants
L="$V/base.so $V/w64.so $V/w64g16.so $V/w64noprio.so"
: > "$OUT/ab_r29.jsonl"
timeout -k 10 300 python tools/kbench.py --n 8 --rounds 20 $L >> "$OUT/ab_r29.jsonl" || exit 1
timeout -k 10 300 python tools/kbench.py --n 8 --rounds 20 $L >> "$OUT/ab_r29.jsonl" || exit 1
cat "$OUT/ab_r29.jsonl"
