#!/bin/bash
# seam-step timing + kernel trace of it
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
timeout -k 10 300 python tools/seam_bench.py --size 16384 --n 8 > "$OUT/seam_bench.jsonl" 2> "$OUT/seam_bench.err"
rc=$?; cat "$OUT/seam_bench.jsonl"; tail -3 "$OUT/seam_bench.err"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/seam_bench.py --size 4096 --n 8 >> "$OUT/seam_bench.jsonl" 2>> "$OUT/seam_bench.err"
rc=$?; tail -1 "$OUT/seam_bench.jsonl"; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof_seam" -o run -- python3 "$GRAFT_REPO_ROOT/tools/seam_bench.py" --size 16384 --n 8 > "$OUT/prof_seam.log" 2>&1
rc=$?; tail -2 "$OUT/prof_seam.log"; grep -E "seam|dcte" "$OUT/prof_seam/run_kernel_stats.csv" | cut -c1-150; exit $rc
