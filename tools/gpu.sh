#!/bin/bash
# One gpurun call, parametrised (replaces the per-run gpu_rNN*.sh one-liners):
#   bash tools/gpu.sh TAG STEP [STEP ...]
# STEP is one of
#   tests              the whole -m gpu suite            -> gpurun_out/TAG/gpu_tests.log
#   tests:ARGS         the -m gpu suite with pytest ARGS -> gpurun_out/TAG/gpu_tests.log
#   bench:ARGS         python bench.py ARGS              -> gpurun_out/TAG/bench[_i].json / .err
#   profile            tools/profile_round.sh TAG        -> gpurun_out/prof_TAG/
#   py:SCRIPT ARGS     python3 -u SCRIPT ARGS            -> gpurun_out/TAG/py[_i].log
# Every step runs under its own time limit; the first failing step ends the call.
set -u
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
i=0
for step in "$@"; do
  i=$((i + 1))
  kind=${step%%:*}
  arg=""
  [[ "$step" == *:* ]] && arg=${step#*:}
  case "$kind" in
    tests)
      # shellcheck disable=SC2086
      timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread $arg \
        > "$OUT/gpu_tests.log" 2>&1
      rc=$?; tail -3 "$OUT/gpu_tests.log" ;;
    bench)
      # shellcheck disable=SC2086
      timeout -k 10 600 python3 -u bench.py $arg > "$OUT/bench_$i.json" 2> "$OUT/bench_$i.err"
      rc=$?; tail -c 600 "$OUT/bench_$i.json" ;;
    profile)
      bash tools/profile_round.sh "$TAG"; rc=$? ;;
    py)
      # shellcheck disable=SC2086
      timeout -k 10 600 python3 -u $arg > "$OUT/py_$i.log" 2>&1
      rc=$?; tail -5 "$OUT/py_$i.log" ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
  if [ $rc -ne 0 ]; then echo "step $i ($step) failed: rc=$rc"; exit $rc; fi
done
echo "all steps done"
