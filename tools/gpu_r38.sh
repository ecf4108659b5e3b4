#!/bin/bash
# Seam DP band height (= halo width) A/B: R = 32 (base), 40, 36 rows per band;
# every variant's seams checked against the oracle, then the seam GPU tests on
# each candidate build.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
V=dct-carver_amd/build/variants
: > "$OUT/ab_r38.jsonl"
for r in 1 2; do
  for v in base r40q5 r36q3 r40q5nb2; do
    timeout -k 10 200 python tools/dp_bench.py --size 16384 --check --lib $V/$v.so >> "$OUT/ab_r38.jsonl" || exit 1
  done
done
cat "$OUT/ab_r38.jsonl"
for v in r40q5 r36q3; do
  DCTE_LIB=$V/$v.so timeout -k 10 600 python -u -m pytest tests/test_seam_dp.py tests/test_seam.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_dp_$v.log" 2>&1
  rc=$?; echo "$v pytest exit $rc"; tail -2 "$OUT/pytest_dp_$v.log"; [ $rc -eq 0 ] || exit $rc
done
