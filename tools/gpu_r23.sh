#!/bin/bash
# XCD-contiguous tile order A/B: time (interleaved, one process) and HBM bytes
# per launch (FETCH_SIZE / WRITE_SIZE passes of the bench on each build).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
export TMPDIR=/tmp
V="$GRAFT_REPO_ROOT/dct-carver_amd/build/variants"
timeout -k 10 300 python tools/kbench.py --n 8 --rounds 7 $V/xcd0.so $V/xcd1.so > "$OUT/ab_r23.jsonl" 2> "$OUT/ab_r23.err" || { echo "ab failed"; tail -5 "$OUT/ab_r23.err"; exit 1; }
cat "$OUT/ab_r23.jsonl"
cd /tmp
for v in xcd0 xcd1; do
  export DCTE_LIB=$V/$v.so
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d "$OUT/xcd_$v/pmc_FETCH_SIZE" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/xcd_$v.log" 2>&1 || { echo "pmc $v failed"; tail -5 "$OUT/xcd_$v.log"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d "$OUT/xcd_$v/pmc_WRITE_SIZE" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline >> "$OUT/xcd_$v.log" 2>&1 || { echo "pmc $v failed"; tail -5 "$OUT/xcd_$v.log"; exit 1; }
done
