#!/bin/bash
# A/B: wave priority raised while a workgroup stages / converts a row group.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
V=dct-carver_amd/build/variants
timeout -k 10 300 python tools/kbench.py --n 8 --rounds 9 $V/base.so $V/prio1.so $V/prio3.so > "$OUT/ab_r24.jsonl" 2> "$OUT/ab_r24.err" || { echo "ab failed"; tail -5 "$OUT/ab_r24.err"; exit 1; }
cat "$OUT/ab_r24.jsonl"
