#!/bin/bash
# Bench at its defaults, the kernel-trace summary of that SAME command (so the
# traced average and the bench's HIP-event average describe the same launches),
# and every-N kernel timings.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo bench failed; tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof_bench" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" > "$OUT/prof_bench.json" 2> "$OUT/prof_bench.err") || { echo "trace failed"; tail -5 "$OUT/prof_bench.err"; exit 1; }
cat "$OUT/prof_bench.json"
bash tools/gpu_nall.sh
