#!/bin/bash
# Rehearsal of the N > 1 bench path on one GPU (gloo halo staging, 2 ranks on
# the same device): weak (default) and strong (--strong) scaling, bands
# recomputed without exchange and required bit-equal (--check).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
: > "$OUT/rehearsal_r34.jsonl"
for mode in "" "--strong"; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
    bench.py --gpus 2 --steps 10 --warmup 3 --dist-backend gloo --check $mode >> "$OUT/rehearsal_r34.jsonl" 2> "$OUT/rehearsal_r34.err" || { tail -20 "$OUT/rehearsal_r34.err"; exit 1; }
done
timeout -k 10 300 python bench.py --strong --steps 10 --warmup 3 --no-cpu-baseline --check >> "$OUT/rehearsal_r34.jsonl" || exit 1
cat "$OUT/rehearsal_r34.jsonl"
