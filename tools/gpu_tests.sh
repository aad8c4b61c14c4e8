#!/bin/bash
# GPU test suite on the box: bash tools/gpu_tests.sh TAG [pytest args...]
set -u
TAG=$1; shift
mkdir -p gpurun_out/$TAG
timeout -k 10 1100 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread "$@" > gpurun_out/$TAG/gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/$TAG/gpu_tests.log
exit $rc
