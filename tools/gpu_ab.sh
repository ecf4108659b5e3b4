#!/bin/bash
# A/B the variant builds (tools/variants.sh) on the GPU, then the GPU tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
V=dct-carver_amd/build/variants
timeout -k 10 300 python tools/kbench.py --n 8 $V/*.so > "$OUT/ab_n8.jsonl" 2> "$OUT/ab_n8.err" || { echo "ab failed"; tail -5 "$OUT/ab_n8.err"; exit 1; }
cat "$OUT/ab_n8.jsonl"
if [ "${RUN_TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
  echo "pytest exit $?" >> "$OUT/pytest_gpu.log"
  tail -4 "$OUT/pytest_gpu.log"
fi
