set -u
O=gpurun_out/r04o; mkdir -p $O
export TMPDIR=/tmp
for P in 2 3 4; do
  SG_PLAN_DIAG=1 SG_SSSP_PHASES=$P timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/p$P -o run -- python3 tools/sssp_one.py > $O/one_$P.log 2>&1 || exit 1
  echo "phases=$P"; grep "\[plan\]" $O/one_$P.log | tail -1
  python3 - $O/p$P <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
ks = [r for r in rows if "k_sssp_lds" in r["Kernel_Name"]]
half = ks[len(ks) // 2:]
print("  second build, launches (us):", [round((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, 1) for r in half])
PY
done
