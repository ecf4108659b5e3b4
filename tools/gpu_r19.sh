#!/bin/bash
# Map kernel A/B (N = 8, 16384^2 RGB): tools/variants.sh builds interleaved in
# one process (bit-equality against the first), then the parity tests that pin
# the fp32 path (device == host emulation, tolerance vs the oracle).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
V=dct-carver_amd/build/variants
timeout -k 10 300 python tools/kbench.py --n 8 --rounds 7 $V/base.so $V/db.so $V/dbx.so $V/p.so $V/dbxp.so > "$OUT/ab_r19.jsonl" 2> "$OUT/ab_r19.err" || { echo "ab failed"; tail -5 "$OUT/ab_r19.err"; exit 1; }
cat "$OUT/ab_r19.jsonl"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_seam.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_r19.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_r19.log"; exit $rc
