set -u
O=gpurun_out/r04k; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python3 tools/sssp_ab.py --reps 9 SG_SSSP_FLAGGED=0 SG_SSSP_FLAGGED=1 "SG_SSSP_FLAGGED=1,SG_SSSP_PHASES=3" "SG_SSSP_FLAGGED=1,SG_SSSP_PHASES=4" > $O/ab_full.log 2>&1 || { tail -5 $O/ab_full.log; exit 1; }
cut -c1-160 $O/ab_full.log
for R in 0:1250 0:2500 0:5000; do
  timeout -k 10 200 python3 tools/sssp_ab.py --reps 9 --rows $R SG_SSSP_FLAGGED=0 SG_SSSP_FLAGGED=1 "SG_SSSP_FLAGGED=1,SG_SSSP_PHASES=3" "SG_SSSP_SEEDS=0" > $O/ab_$R.log 2>&1 || { tail -5 $O/ab_$R.log; exit 1; }
  echo "rows $R"; cut -c1-160 $O/ab_$R.log
done
timeout -k 10 200 python3 tools/round_c5.py --rounds 8 > $O/c5.log 2>&1 || { tail -5 $O/c5.log; exit 1; }
tail -3 $O/c5.log
timeout -k 10 200 python3 tools/round_c5.py --rounds 20 --nodes 10000 --hosts 100000 --packets 1000000 > $O/c4.log 2>&1 || { tail -5 $O/c4.log; exit 1; }
tail -3 $O/c4.log
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --durations=40 > $O/tests.log 2>&1; rc=$?
tail -60 $O/tests.log | head -50
exit $rc
