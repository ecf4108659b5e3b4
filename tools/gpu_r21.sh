#!/bin/bash
# Round-end refresh: all GPU tests, smoke, bench, seam-loop / DP timing,
# kernel-trace stats (bench and carve loop), PMC passes over the bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest exit $rc" >> "$OUT/pytest_gpu.log"; tail -3 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo smoke failed; cat "$OUT/smoke.log"; exit 1; }
timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo bench failed; tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
: > "$OUT/seam_loop.jsonl"
timeout -k 10 200 python tools/seam_bench.py --size 4096 --seams 20 --inplace --find >> "$OUT/seam_loop.jsonl" || exit 1
timeout -k 10 200 python tools/seam_bench.py --size 16384 --seams 20 --inplace --find >> "$OUT/seam_loop.jsonl" || exit 1
timeout -k 10 200 python tools/dp_bench.py --size 16384 --check >> "$OUT/seam_loop.jsonl" || exit 1
timeout -k 10 200 python tools/dp_bench.py --size 4096 --check >> "$OUT/seam_loop.jsonl" || exit 1
cat "$OUT/seam_loop.jsonl"
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof_trace" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" > "$OUT/prof_trace.json" 2> "$OUT/prof_trace.log" || { echo "trace failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof_loop" -o run -- python3 "$GRAFT_REPO_ROOT/tools/seam_bench.py" --size 16384 --seams 10 --inplace --find > "$OUT/prof_loop.log" 2>&1 || { echo "loop trace failed"; exit 1; }
for pmc in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_ANY"; do
  tag=$(echo $pmc | tr ' ' '_')
  timeout -s KILL 300 rocprofv3 --pmc $pmc -f csv -d "$OUT/pmc_$tag" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/pmc_$tag.log" 2>&1 || { echo "pmc $pmc failed"; tail -5 "$OUT/pmc_$tag.log"; exit 1; }
done
find "$OUT" -name "*stats.csv"
