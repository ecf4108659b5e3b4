#!/bin/bash
# bench at N=1 (+check), the N=2 rehearsal on one GPU (gloo halos), trace profile
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --check > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo bench failed; tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --size 4096 --steps 5 --warmup 2 --dist-backend gloo --check --no-cpu-baseline > "$OUT/bench_n2_rehearsal.json" 2> "$OUT/bench_n2.err" || { echo "n2 rehearsal failed"; tail -30 "$OUT/bench_n2.err"; exit 1; }
cat "$OUT/bench_n2_rehearsal.json"
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof_trace" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/prof_trace.log" 2>&1 || { echo "trace failed"; exit 1; }
head -6 "$OUT/prof_trace/run_kernel_stats.csv"
