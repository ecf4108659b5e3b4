#!/bin/bash
# A/B: map-kernel workgroup width for N <= 8 (DCTE_WG8 = 256 / 128 / 64 threads,
# tile_h 128 / 256), interleaved in one process per N; outputs bit-compared.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
V=dct-carver_amd/build/variants
L="$V/base.so $V/w64.so $V/w64t256.so $V/w128.so $V/w128t256.so"
: > "$OUT/ab_r28.jsonl"
timeout -k 10 300 python tools/kbench.py --n 8 --rounds 7 $L >> "$OUT/ab_r28.jsonl" || exit 1
timeout -k 10 300 python tools/kbench.py --n 4 --rounds 5 $L >> "$OUT/ab_r28.jsonl" || exit 1
timeout -k 10 300 python tools/kbench.py --n 8 --sem 1 --rounds 5 $L >> "$OUT/ab_r28.jsonl" || exit 1
cat "$OUT/ab_r28.jsonl"
