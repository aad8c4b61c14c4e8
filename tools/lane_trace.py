import csv, glob, json, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
for name in ("k_inbound", "k_codel<", "k_outbound"):
    ds = [((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, r["Kernel_Name"][:60]) for r in rows if name in r["Kernel_Name"]]
    print(name, [round(d, 1) for d, _ in ds])
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
for k in ("codel", "inbound", "outbound"):
    print(k, "event avg_launch_ms", d[k]["roofline"]["avg_launch_ms"])
