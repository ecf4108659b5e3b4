#!/bin/bash
# N = 8 map kernel: tile height 128/192/224/256/320 rows
# A/B, interleaved, outputs bit-compared.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
V=dct-carver_amd/build/variants
L="$V/base.so $V/th192.so $V/th224.so $V/th256.so $V/th320.so"
: > "$OUT/ab_r40.jsonl"
timeout -k 10 300 python tools/kbench.py --n 8 --rounds 15 $L >> "$OUT/ab_r40.jsonl" || exit 1
timeout -k 10 300 python tools/kbench.py --n 8 --rounds 15 $L >> "$OUT/ab_r40.jsonl" || exit 1
cat "$OUT/ab_r40.jsonl"
