#!/bin/bash
# GPU suite + host-path timing (pinning variants)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest exit $rc" >> "$OUT/pytest_gpu.log"; tail -15 "$OUT/pytest_gpu.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/host_path.py --size 16384 > "$OUT/host_path.jsonl" 2> "$OUT/host_path.err"
rc=$?; cat "$OUT/host_path.jsonl"; tail -3 "$OUT/host_path.err"; exit $rc
