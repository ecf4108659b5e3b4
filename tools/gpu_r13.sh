#!/bin/bash
# seam tests, GPU suite, seam-step timing (copy + in place) + kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
timeout -k 10 300 python -m pytest tests/test_seam.py -m gpu -q -x -p no:cacheprovider > "$OUT/pytest_seam.log" 2>&1
rc=$?; echo "seam exit $rc" >> "$OUT/pytest_seam.log"; tail -25 "$OUT/pytest_seam.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest exit $rc" >> "$OUT/pytest_gpu.log"; tail -3 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
: > "$OUT/seam_bench.jsonl"
for args in "--size 16384" "--size 16384 --inplace" "--size 4096" "--size 4096 --inplace"; do
  timeout -k 10 300 python tools/seam_bench.py --n 8 $args >> "$OUT/seam_bench.jsonl" 2>> "$OUT/seam_bench.err" || { tail -3 "$OUT/seam_bench.err"; exit 1; }
done
cat "$OUT/seam_bench.jsonl"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof_seam" -o run -- python3 "$GRAFT_REPO_ROOT/tools/seam_bench.py" --size 16384 --n 8 --inplace > "$OUT/prof_seam.log" 2>&1
rc=$?; grep -E "seam|dcte" "$OUT/prof_seam/run_kernel_stats.csv" | cut -c1-150; exit $rc
