#!/bin/bash
# AMDGPU machine-scheduler strategy A/B (default / max-ilp / max-memory-clause /
# iterative-ilp) for the N = 8 and N = 16 map kernels, interleaved, bit-compared.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
V=dct-carver_amd/build/variants
L="$V/base.so $V/milp.so $V/mmc.so $V/iilp.so"
: > "$OUT/ab_r43.jsonl"
timeout -k 10 300 python tools/kbench.py --n 8 --rounds 15 $L >> "$OUT/ab_r43.jsonl" || exit 1
timeout -k 10 300 python tools/kbench.py --n 16 --size 8192 --rounds 10 $L >> "$OUT/ab_r43.jsonl" || exit 1
timeout -k 10 300 python tools/kbench.py --n 8 --rounds 15 $L >> "$OUT/ab_r43.jsonl" || exit 1
cat "$OUT/ab_r43.jsonl"
