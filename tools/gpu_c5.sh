# C5 evidence: bench.py --config c5 (50k-node build, 10M-packet round, lane legs at C5 volume,
# the 6,250-row rank block of an 8-way split) under a kernel-trace stats run.
# usage (GPU box): bash tools/gpu_c5.sh TAG
set -u
TAG=$1
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py --config c5 --no-cpu --no-gml --no-c2 --steps 3 --warmup 1 --rank-blocks 8 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 - $O <<'PY'
import csv, glob, json, sys
o = sys.argv[1]
d = json.loads(open(o + "/bench.json").read().strip().splitlines()[-1])
print("value", d["value"], "apsp rank_block", d["apsp_detail"].get("rank_block_ms"))
for k in ("delivery", "codel", "inbound", "outbound"):
    r = d.get(k, {})
    print(k, r.get("ms_per_round", r.get("ms_per_batch", r.get("ms_per_window"))), (r.get("roofline") or {}).get("frac"), (r.get("roofline") or {}).get("avg_launch_ms"))
f = glob.glob(o + "/prof/**/*kernel_stats.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:25]:
    print(f"{r['Name'][:70]:70s} calls {r['Calls']:>5s} avg_us {float(r['AverageNs']) / 1e3:10.2f}")
PY
