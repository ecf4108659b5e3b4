#!/bin/bash
# PMC pass over the DP kernel (dp_bench, default lib)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_MISC -f csv -d "$OUT/pmc_dp" -o run -- python3 "$GRAFT_REPO_ROOT/tools/dp_bench.py" --size 16384 --reps 3 > "$OUT/pmc_dp.log" 2>&1 || { tail -5 "$OUT/pmc_dp.log"; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_IFETCH SQ_ACTIVE_INST_FLAT SQ_WAVES -f csv -d "$OUT/pmc_dp2" -o run -- python3 "$GRAFT_REPO_ROOT/tools/dp_bench.py" --size 16384 --reps 3 > "$OUT/pmc_dp2.log" 2>&1 || { tail -5 "$OUT/pmc_dp2.log"; exit 1; }
find "$OUT" -name "*counter_collection.csv" | head
