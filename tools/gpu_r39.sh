#!/bin/bash
# N = 8 map kernel on the scaled-form passes: tile height (96/128/160/192 rows)
# and staging group (8/16 rows) A/B, interleaved, outputs bit-compared.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
V=dct-carver_amd/build/variants
L="$V/base.so $V/th96.so $V/th160.so $V/th192.so $V/g16.so"
: > "$OUT/ab_r39.jsonl"
timeout -k 10 300 python tools/kbench.py --n 8 --rounds 15 $L >> "$OUT/ab_r39.jsonl" || exit 1
timeout -k 10 300 python tools/kbench.py --n 8 --rounds 15 $L >> "$OUT/ab_r39.jsonl" || exit 1
cat "$OUT/ab_r39.jsonl"
