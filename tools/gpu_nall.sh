#!/bin/bash
# kernel timings for every N on the base build (A/B harness, one process each)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
L=${LIBS:-dct-carver_amd/build/libdctenergy_hip.so}
: > "$OUT/nall.jsonl"
for cfg in "16 8192" "8 16384" "4 16384" "2 16384"; do
  set -- $cfg
  timeout -k 10 300 python tools/kbench.py --n $1 --size $2 $L >> "$OUT/nall.jsonl" 2>> "$OUT/nall.err" || { echo "kbench n=$1 failed"; tail -5 "$OUT/nall.err"; exit 1; }
done
cat "$OUT/nall.jsonl"
