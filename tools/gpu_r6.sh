# Round-6 evidence steps on the GPU box (each GPU step under its own time limit, chained with &&).
# usage: bash tools/gpu_r6.sh TAG STEP...   steps: tests smoke bench c5bench rccl5
set -u
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
for step in "$@"; do
  case $step in
    tests) timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }; tail -3 $O/gpu_tests.log ;;
    c5tests) timeout -k 10 400 python -u -m pytest tests/test_c5_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/c5_tests.log 2>&1 || { tail -30 $O/c5_tests.log; exit 1; }; tail -12 $O/c5_tests.log ;;
    smoke) timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }; tail -2 $O/smoke.log ;;
    bench) timeout -k 10 420 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }; tail -c 600 $O/bench.json ;;
    c5bench) timeout -k 10 600 python -u bench.py --config c5 --no-gml --no-c2 --steps 3 --warmup 1 --rank-blocks 8 > $O/bench_c5.json 2> $O/bench_c5.err || { tail -20 $O/bench_c5.err; exit 1; }; tail -c 400 $O/bench_c5.json ;;
    rccl5) MASTER_PORT=29561 timeout -k 10 300 python -u tools/rccl_check.py --c5 --reps 5 > $O/rccl_c5.json 2> $O/rccl_c5.err || { tail -20 $O/rccl_c5.err; exit 1; }; tail -c 800 $O/rccl_c5.json ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
