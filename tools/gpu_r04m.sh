set -u
O=gpurun_out/r04m; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_deliver_gpu.py tests/test_c5_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for L in tools/ab/libshadow_gpu_r03.so ""; do
  N=$(basename ${L:-head})
  if [ -n "$L" ]; then export SHADOW_GPU_LIB=$L; else unset SHADOW_GPU_LIB; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_$N -o run -- python3 tools/round_c5.py --rounds 8 > $O/c5_$N.log 2>&1 || exit 1
  echo "lib=$N"; tail -2 $O/c5_$N.log
  python3 - $O/p_$N <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "sg::" in r["Name"] and "table_pack" not in r["Name"]:
        print(f"  {r['Name'][:64]:64s} {r['Calls']:>4s} {float(r['AverageNs']) / 1e3:9.2f}")
PY
done
unset SHADOW_GPU_LIB
timeout -k 10 200 python3 tools/round_c5.py --rounds 12 > $O/c5_head_noprof.log 2>&1 || exit 1
tail -3 $O/c5_head_noprof.log
