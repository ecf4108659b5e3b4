#!/bin/bash
# GPU pass: parity tests, smoke, bench, kernel-trace stats (csv), PMC passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
rc=$?
echo "pytest exit $rc" >> "$OUT/pytest_gpu.log"
tail -3 "$OUT/pytest_gpu.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest crashed ($rc)"; exit 1; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo smoke failed; cat "$OUT/smoke.log"; exit 1; }
timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo bench failed; tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
cd /tmp
rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof_trace" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/prof_trace.log" 2>&1 || { echo "trace failed"; exit 1; }
for pmc in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_ANY"; do
  tag=$(echo $pmc | tr ' ' '_')
  timeout -k 10 400 rocprofv3 --pmc $pmc -f csv -d "$OUT/pmc_$tag" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/pmc_$tag.log" 2>&1 || { echo "pmc $pmc failed"; tail -5 "$OUT/pmc_$tag.log"; exit 1; }
done
find "$OUT" -name "*.csv" | head -20
