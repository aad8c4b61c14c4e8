# C4 round A/B: the delivery GPU tests, tools/round_c4.py, and its kernel-trace stats.
# usage (GPU box): bash tools/gpu_c4.sh TAG [ENV_SETTING ...] (settings as tools/round_c4.py takes them)
set -u
TAG=$1
shift
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_deliver_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -u tools/round_c4.py "$@" > $O/round.log 2>&1 || { tail -5 $O/round.log; exit 1; }
cat $O/round.log
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/round_c4.py > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
python3 - $O/prof <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(f"{r['Name'][:60]:60s} calls {r['Calls']:>5s} avg_us {float(r['AverageNs']) / 1e3:8.2f}")
PY
