set -u
O=gpurun_out/r04l; mkdir -p $O
export TMPDIR=/tmp
for L in tools/ab/libshadow_gpu_r03.so tools/ab/libshadow_gpu_r04bitonic.so ""; do
  if [ -n "$L" ]; then export SHADOW_GPU_LIB=$L; else unset SHADOW_GPU_LIB; fi
  echo "lib=${L:-head}"
  timeout -k 10 200 python3 tools/round_c5.py --rounds 12 > $O/c5_$(basename ${L:-head}).log 2>&1 || exit 1
  tail -4 $O/c5_$(basename ${L:-head}).log
done
unset SHADOW_GPU_LIB
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/round_c5.py --rounds 6 > $O/prof.log 2>&1 || exit 1
python3 - $O/prof <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(f"{r['Name'][:70]:70s} {r['Calls']:>4s} {float(r['AverageNs']) / 1e3:9.2f}")
PY
