set -u
O=gpurun_out/r04p; mkdir -p $O
export TMPDIR=/tmp
SG_PLAN_DIAG=1 timeout -k 10 300 python3 tools/sssp_ab.py --reps 9 SG_SSSP_HOP0=1 SG_SSSP_HOP0=2 "SG_SSSP_HOP0=2,SG_SSSP_PHASES=4" "SG_SSSP_HOP0=3,SG_SSSP_PHASES=4" "SG_SSSP_HOP0=3,SG_SSSP_PHASES=5" "SG_SSSP_HOP0=2,SG_SSSP_BOUNDS=3" > $O/ab.log 2> $O/ab.err || { tail -5 $O/ab.err; exit 1; }
cut -c1-220 $O/ab.log; grep "\[plan\]" $O/ab.err | sort | uniq -c
for V in "2 3" "2 4" "3 4"; do
  set -- $V
  SG_SSSP_HOP0=$1 SG_SSSP_PHASES=$2 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/p$1_$2 -o run -- python3 tools/sssp_one.py > $O/one_$1_$2.log 2>&1 || exit 1
  python3 - $O/p$1_$2 "$V" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
ks = [r for r in rows if "k_sssp_lds" in r["Kernel_Name"]]
half = ks[len(ks) // 2:]
print("hop0/phases", sys.argv[2], "second build, launches (us):", [round((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, 1) for r in half])
PY
done
