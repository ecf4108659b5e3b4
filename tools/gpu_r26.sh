#!/bin/bash
# A/B: seam compaction chunk per thread (dwords per pass), in-place carve step at
# 16384^2 RGB (seams given: compaction + band update only), then with the search.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
V="$GRAFT_REPO_ROOT/dct-carver_amd/build/variants"
: > "$OUT/ab_r26.jsonl"
for r in 1 2; do
  for v in sh4 sh8 sh16; do
    DCTE_LIB=$V/$v.so timeout -k 10 120 python tools/seam_bench.py --size 16384 --seams 20 --inplace | sed "s/^{/{\"lib\": \"$v\", /" >> "$OUT/ab_r26.jsonl" || exit 1
  done
done
cat "$OUT/ab_r26.jsonl"
