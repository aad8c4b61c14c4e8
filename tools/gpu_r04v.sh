# queue-ahead event timing in bench.py (lane and walk rooflines vs rocprof), the fill test trim
set -u
O=gpurun_out/r04v; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_routing_gpu.py -m gpu -q -k fill_c3 --timeout 120 --timeout-method thread > $O/fill.log 2>&1
rc=$?; tail -2 $O/fill.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u bench.py --no-cpu > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 - $O/bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", d["value"], "frac", d["roofline"]["frac"], d["roofline"]["avg_launch_ms"])
for k in ("delivery", "codel", "inbound", "outbound", "c2"):
    r = d.get(k, {}).get("roofline")
    if r: print(k, r["avg_launch_ms"], r["frac"], r.get("rocprof"))
print("kernel_ms", d["delivery"].get("kernel_ms"))
PY
