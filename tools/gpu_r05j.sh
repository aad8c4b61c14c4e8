# nontemporal cell gather in k_walk: C4 round time and FETCH_SIZE, default vs variant library
set -u
export TMPDIR=/tmp
O=gpurun_out/r05j; mkdir -p $O
timeout -k 10 120 python3 -u tools/round_c4.py "" > $O/def.log 2>&1 && cat $O/def.log | grep round
SHADOW_GPU_LIB=$PWD/tools/ab/libshadow_gpu_ntcell.so timeout -k 10 120 python3 -u tools/round_c4.py "" > $O/nt.log 2>&1 && cat $O/nt.log | grep round
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f_def -o run -- python3 tools/round_c4.py "" > $O/f_def.log 2>&1 || exit 1
SHADOW_GPU_LIB=$PWD/tools/ab/libshadow_gpu_ntcell.so timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f_nt -o run -- python3 tools/round_c4.py "" > $O/f_nt.log 2>&1 || exit 1
python3 - $O <<'PY'
import csv, glob, sys, collections
for v in ("f_def", "f_nt"):
    acc = collections.defaultdict(list)
    for f in glob.glob(sys.argv[1] + "/" + v + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_walk" in r["Kernel_Name"]:
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(v, {k: sum(x) / len(x) for k, x in acc.items()})
PY
