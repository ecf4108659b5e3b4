#!/bin/bash
# DP: parity tests, then DP-only timing of the default build and variants at 16384^2
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
timeout -k 10 300 python -m pytest tests/test_seam_dp.py -m gpu -q -x -p no:cacheprovider > "$OUT/pytest_dp.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_dp.log"; [ $rc -eq 0 ] || exit $rc
: > "$OUT/dp_var.jsonl"
timeout -k 10 120 python tools/dp_bench.py --size 16384 --check >> "$OUT/dp_var.jsonl" || exit 1
timeout -k 10 120 python tools/dp_bench.py --size 4096 --check >> "$OUT/dp_var.jsonl" || exit 1
for v in nb8 nodpp nosrc pure pure_nosrc; do
  timeout -k 10 120 python tools/dp_bench.py --size 16384 --check --lib dct-carver_amd/build/variants/$v.so >> "$OUT/dp_var.jsonl" || exit 1
done
cat "$OUT/dp_var.jsonl"
