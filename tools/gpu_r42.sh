#!/bin/bash
# N = 16 map kernel (8192^2 RGB): tile height 64/128/192/256 rows, interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
V=dct-carver_amd/build/variants
L="$V/base.so $V/t64.so $V/t192.so $V/t256.so"
: > "$OUT/ab_r42.jsonl"
timeout -k 10 300 python tools/kbench.py --n 16 --size 8192 --rounds 15 $L >> "$OUT/ab_r42.jsonl" || exit 1
timeout -k 10 300 python tools/kbench.py --n 16 --size 8192 --rounds 15 $L >> "$OUT/ab_r42.jsonl" || exit 1
cat "$OUT/ab_r42.jsonl"
