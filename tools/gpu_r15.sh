#!/bin/bash
# seam DP v2 (DPP, tagged hand-off): tests, full GPU suite, carve-loop timing + kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
timeout -k 10 300 python -m pytest tests/test_seam_dp.py -m gpu -q -x -p no:cacheprovider > "$OUT/pytest_dp.log" 2>&1
rc=$?; echo "dp exit $rc" >> "$OUT/pytest_dp.log"; tail -25 "$OUT/pytest_dp.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest exit $rc" >> "$OUT/pytest_gpu.log"; tail -3 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
: > "$OUT/seam_loop.jsonl"
for args in "--size 4096" "--size 16384"; do
  timeout -k 10 300 python tools/seam_bench.py --n 8 --inplace --find $args >> "$OUT/seam_loop.jsonl" 2>> "$OUT/seam_loop.err" || { tail -3 "$OUT/seam_loop.err"; exit 1; }
done
cat "$OUT/seam_loop.jsonl"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof_loop" -o run -- python3 "$GRAFT_REPO_ROOT/tools/seam_bench.py" --size 16384 --n 8 --inplace --find > "$OUT/prof_loop.log" 2>&1
rc=$?; grep -E "seam|dcte" "$OUT/prof_loop/run_kernel_stats.csv" | cut -c1-150; exit $rc
