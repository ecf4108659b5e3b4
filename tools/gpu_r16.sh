#!/bin/bash
# DP v3: tests + DP-only timing (default vs no-exchange variant)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
timeout -k 10 300 python -m pytest tests/test_seam_dp.py -m gpu -q -x -p no:cacheprovider > "$OUT/pytest_dp.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_dp.log"; [ $rc -eq 0 ] || exit $rc
: > "$OUT/dp_bench.jsonl"
for s in 4096 16384; do
  timeout -k 10 120 python tools/dp_bench.py --size $s --check >> "$OUT/dp_bench.jsonl" || exit 1
  timeout -k 10 120 python tools/dp_bench.py --size $s --lib dct-carver_amd/build/variants/noxch.so >> "$OUT/dp_bench.jsonl" || exit 1
done
cat "$OUT/dp_bench.jsonl"
