#!/bin/bash
# One parameterised GPU runner (replaces the per-session tools/gpu_r*.sh).
#
#   gpurun -- tools/gpu.sh STEP [STEP ...]
#
# STEP is NAME or NAME:ARGS (ARGS one quoted word, word-split by the shell, so
# inner quotes group: tests:"-k 'refine or stress'"):
#   tests[:PYTEST-ARGS]    pytest -m gpu -s (e.g. tests:"-k full_frame")
#   smoke                  __graft_entry__.smoke()
#   bench[:ARGS]           python bench.py ARGS          -> NN_bench.json
#   trace[:ARGS]           rocprofv3 --kernel-trace --stats of bench.py ARGS
#   pmc:CTRS[:ARGS]        one rocprofv3 --pmc pass, CTRS comma-separated
#   py:SCRIPT ARGS         python SCRIPT ARGS (tools/kbench.py, tools/*.py)
#   ptrace:SCRIPT ARGS     rocprofv3 --kernel-trace --stats of python3 SCRIPT ARGS
#   ppmc:CTRS:SCRIPT ARGS  one rocprofv3 --pmc pass over python3 SCRIPT ARGS
# Every step runs under its own time limit (STEP_TIMEOUT, default 300 s;
# tests 900 s) and the script stops at the first failing step: after a fault,
# an abort or a time limit nothing else touches the GPU.  Output goes to
# gpurun_out/NN_NAME.{log,json} and rocprof data to gpurun_out/NN_NAME/.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
export TMPDIR=/tmp
T=${STEP_TIMEOUT:-300}
i=0
for step in "$@"; do
  i=$((i + 1))
  name=${step%%:*}
  args=""
  [ "$step" != "$name" ] && args=${step#*:}
  tag=$(printf "%02d_%s" $i "$name")
  echo "== step $tag: $args"
  case "$name" in
    tests)
      eval "timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread \
        -p no:cacheprovider $args" > "$OUT/$tag.log" 2>&1
      rc=$?; tail -5 "$OUT/$tag.log" ;;
    smoke)
      timeout -k 10 "$T" python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/$tag.log" 2>&1
      rc=$?; tail -2 "$OUT/$tag.log" ;;
    bench)
      eval "timeout -k 10 $T python bench.py $args" > "$OUT/$tag.json" 2> "$OUT/$tag.log"
      rc=$?; cat "$OUT/$tag.json"; [ $rc -eq 0 ] || tail -20 "$OUT/$tag.log" ;;
    trace)
      (cd /tmp && timeout -k 10 "$T" rocprofv3 --kernel-trace --stats -f csv -d "$OUT/$tag" -o run \
        -- python3 "$GRAFT_REPO_ROOT/bench.py" $args > "$OUT/$tag.log" 2>&1)
      rc=$?; tail -3 "$OUT/$tag.log" ;;
    pmc)
      ctrs=${args%%:*}
      rest=""
      [ "$args" != "$ctrs" ] && rest=${args#*:}
      (cd /tmp && timeout -k 10 -s KILL 120 rocprofv3 --pmc ${ctrs//,/ } -f csv -d "$OUT/$tag" -o run \
        -- python3 "$GRAFT_REPO_ROOT/bench.py" $rest > "$OUT/$tag.log" 2>&1)
      rc=$?; tail -3 "$OUT/$tag.log" ;;
    ptrace)
      (cd /tmp && eval "timeout -k 10 $T rocprofv3 --kernel-trace --stats -f csv -d $OUT/$tag -o run \
        -- python3 $GRAFT_REPO_ROOT/$args" > "$OUT/$tag.log" 2>&1)
      rc=$?; tail -3 "$OUT/$tag.log" ;;
    ppmc)
      ctrs=${args%%:*}
      rest=${args#*:}
      (cd /tmp && eval "timeout -k 10 -s KILL 120 rocprofv3 --pmc ${ctrs//,/ } -f csv -d $OUT/$tag -o run \
        -- python3 $GRAFT_REPO_ROOT/$rest" > "$OUT/$tag.log" 2>&1)
      rc=$?; tail -3 "$OUT/$tag.log" ;;
    py)
      eval "timeout -k 10 $T python -u $args" > "$OUT/$tag.log" 2>&1
      rc=$?; tail -40 "$OUT/$tag.log" ;;
    *)
      echo "unknown step $name"; exit 2 ;;
  esac
  echo "== step $tag exit $rc"
  [ $rc -eq 0 ] || exit $rc
done
