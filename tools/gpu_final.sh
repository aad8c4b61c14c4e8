# Final evidence for a round (one gpurun call): the whole -m gpu suite, the default bench line,
# the rocprof summaries (profile_round.sh), and an N=2 gloo rehearsal of the N-rank bench path
# (both ranks on this box's one card: host-staged collectives, so its times are not measurements).
# usage: bash tools/gpu_final.sh TAG
set -u
TAG=$1
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread --durations=15 > $O/gpu_tests.log 2>&1
rc=$?; tail -2 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python3 -u bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
tail -c 300 $O/bench.json
bash tools/profile_round.sh $TAG || exit 1
SG_BENCH_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu --no-gml --no-c2 \
  > $O/bench_n2_gloo.json 2> $O/bench_n2_gloo.err || { tail -5 $O/bench_n2_gloo.err; exit 1; }
tail -c 200 $O/bench_n2_gloo.json
echo final done
