set -u
O=gpurun_out/r8j; mkdir -p $O
export TMPDIR=/tmp
for l in base wnt wb0 wb1 wb2 wb16 wb17; do
  if [ $l = base ]; then L=shadow_amd/libshadow_gpu.so; else L=tools/ab/libshadow_gpu_$l.so; fi
  [ -f $L ] || { echo missing $L; exit 1; }
  SHADOW_GPU_LIB=$L timeout -k 10 120 python3 -u tools/round_c4.py > $O/t_$l.log 2>&1 || { tail -5 $O/t_$l.log; exit 1; }
  SHADOW_GPU_LIB=$L timeout -s KILL 120 rocprofv3 --kernel-include-regex k_walk --pmc FETCH_SIZE --output-format csv -d $O/p_$l -o run -- python3 tools/round_c4.py > $O/p_$l.log 2>&1 || { echo "pmc $l failed"; tail -5 $O/p_$l.log; exit 1; }
  F=$(python3 -c "
import csv,glob
v=[float(r['Counter_Value']) for f in glob.glob('$O/p_$l/**/*counter_collection.csv',recursive=True) for r in csv.DictReader(open(f)) if r['Counter_Name']=='FETCH_SIZE']
print(round(sum(v)/len(v)), len(v))")
  echo "$l: $(grep round $O/t_$l.log) fetch_kb $F"
done
