# timing events without the system-scope fence: the bench line's event averages against rocprof
set -u
O=gpurun_out/r05zb; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u bench.py --no-cpu --no-gml > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 - $O/bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", d["value"], "apsp", d["roofline"]["avg_launch_ms"], d["roofline"]["frac"], d["roofline"].get("rocprof"))
for k in ("delivery", "codel", "inbound", "outbound", "c2"):
    r = d[k]["roofline"]; print(k, r["avg_launch_ms"], r["frac"], r.get("rocprof"))
print(d["delivery"]["kernel_ms"], d["delivery"]["ms_per_round"])
PY
