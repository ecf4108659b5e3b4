#!/bin/bash
# Re-check of the N = 8 tuning knobs on the scaled-form kernel: staging priority,
# halo-conversion balancing, XCD tile order (N = 8 and N = 16), interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
V=dct-carver_amd/build/variants
L="$V/base.so $V/prio0.so $V/xbal0.so $V/xcd0.so"
: > "$OUT/ab_r44.jsonl"
timeout -k 10 300 python tools/kbench.py --n 8 --rounds 15 $L >> "$OUT/ab_r44.jsonl" || exit 1
timeout -k 10 300 python tools/kbench.py --n 16 --size 8192 --rounds 10 $L >> "$OUT/ab_r44.jsonl" || exit 1
timeout -k 10 300 python tools/kbench.py --n 8 --rounds 15 $L >> "$OUT/ab_r44.jsonl" || exit 1
cat "$OUT/ab_r44.jsonl"
