#!/bin/bash
# Map kernel A/B round 2 (tile height, group size, occupancy bound) + the seam
# DP / host-carve tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
V=dct-carver_amd/build/variants
timeout -k 10 300 python tools/kbench.py --n 8 --rounds 7 $V/dbxp.so $V/g16.so $V/t256.so $V/t64.so $V/mw2.so > "$OUT/ab_r20.jsonl" 2> "$OUT/ab_r20.err" || { echo "ab failed"; tail -5 "$OUT/ab_r20.err"; exit 1; }
cat "$OUT/ab_r20.jsonl"
timeout -k 10 600 python -u -m pytest tests/test_seam_dp.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_r20.log" 2>&1
rc=$?; tail -5 "$OUT/pytest_r20.log"; exit $rc
