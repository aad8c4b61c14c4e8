#!/usr/bin/env python3
"""Summarise rocprofv3 output into profiles/ JSON.

  kernel stats : rocprofv3 --kernel-trace --stats --output-format csv -d DIR -- python bench.py ...
  PMC passes   : rocprofv3 --pmc FETCH_SIZE  --output-format csv -d DIR_F -- python bench.py ...
                 rocprofv3 --pmc WRITE_SIZE  --output-format csv -d DIR_W -- python bench.py ...

    python tools/pmc_summary.py --stats DIR --fetch DIR_F --write DIR_W -o profiles/pmc_r01.json

Per kernel: average FETCH_SIZE / WRITE_SIZE per dispatch (rocprofv3 reports KB),
HBM bytes per launch = (FETCH_SIZE * 2 + WRITE_SIZE) * 1024, where the x2 is the
gfx950 correction of MI355X_MICROARCH.md §HBM (FETCH_SIZE reads half the bytes of
a wide coalesced stream; calibrated for 16-B/lane loads -- our 8-B/lane gathers
are uncalibrated, so the raw value is kept beside it).
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

# first match wins: k_relax_wide before the k_relax<...> template instances
KERNELS = {"relax_wide": "k_relax_wide", "sssp_fill": "k_sssp_lds<false, 1024, 8, 1, false>",
           "sssp_fill_flagged": "k_sssp_lds<false, 1024, 8, 1, true>",
           "sssp_count": "k_sssp_lds<true", "sssp": "k_sssp_lds<false, 1024, 8, 0, false>",
           "sssp_flagged": "k_sssp_lds<false, 1024, 8, 0, true>", "relax": "k_relax_w2<", "relax1": "k_relax_w<", "out": "k_out_batch", "walk": "k_walk",
           "sb_hist": "k_sb_hist", "sb_scatter": "k_sb_scatter", "sb_sort_region": "k_sb_sort_region",
           "sb_sort": "k_sb_sort", "sort_big": "k_sort_big", "host_off": "k_host_off", "reduce_stats": "k_reduce_stats",
           "table_pack": "k_table_pack", "codel_reduce": "k_codel_reduce", "codel": "k_codel",
           "inbound": "k_inbound",
           "outbound": "k_outbound",
           "out_compact": "k_out_compact",
           "sssp_dense": "k_sssp_dense", "dense_sort": "k_sort_arcs",
           "sssp_band": "k_sssp_band<false", "sssp_bucket": "k_sssp_bucket<false",
           "init": "k_init_batch"}
VALU_PEAK_OPS_PER_NS = 256 * 4 * 32 * 2.4  # 78.6e3 lane-ops per ns (MI355X_MICROARCH.md chip table)


def _rows(d, pattern):
    out = []
    for f in glob.glob(os.path.join(d, "**", pattern), recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def short(name):
    for k, v in KERNELS.items():
        if v in name:
            return k
    return None


def counter_avgs(d, counter, agg=None):
    """Average per dispatch of the most-dispatched instantiation of each kernel
    (bench's one work-counting run uses another template instance); agg=max: its largest
    dispatch (a kernel launched at several sizes, e.g. k_sssp_band's one-shot build beside
    the row blocks of bench's rank-block leg)."""
    acc = defaultdict(lambda: defaultdict(list))
    for r in _rows(d, "*counter_collection.csv"):
        if r.get("Counter_Name") != counter:
            continue
        name = r.get("Kernel_Name", "")
        k = short(name)
        if k:
            acc[k][name].append(float(r["Counter_Value"]))
    out = {}
    for k, by_name in acc.items():
        vals = max(by_name.values(), key=len)
        out[k] = agg(vals) if agg else sum(vals) / len(vals)
    return out


def stats(d):
    res = {}
    for r in _rows(d, "*kernel_stats.csv"):
        k = short(r.get("Name", ""))
        if k and (k not in res or int(r["Calls"]) > res[k]["calls"]):
            res[k] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]), "total_ns": float(r["TotalDurationNs"]),
                      "max_ns": float(r.get("MaxNs", 0) or 0), "pct": float(r.get("Percentage", 0) or 0)}
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stats")
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--sq", help="pass with SQ_INSTS_VALU (VALU utilisation)")
    ap.add_argument("-o", "--out", required=True)
    a = ap.parse_args()
    out = {}
    st = stats(a.stats) if a.stats else {}
    fe = counter_avgs(a.fetch, "FETCH_SIZE") if a.fetch else {}
    wr = counter_avgs(a.write, "WRITE_SIZE") if a.write else {}
    va = counter_avgs(a.sq, "SQ_INSTS_VALU") if a.sq else {}
    fe_mx = counter_avgs(a.fetch, "FETCH_SIZE", max) if a.fetch else {}
    wr_mx = counter_avgs(a.write, "WRITE_SIZE", max) if a.write else {}
    va_mx = counter_avgs(a.sq, "SQ_INSTS_VALU", max) if a.sq else {}
    for k in sorted(set(st) | set(fe) | set(wr) | set(va)):
        e = {}
        if k in st:
            e.update(st[k])
        if k in fe:
            e["fetch_kb_raw"] = fe[k]
        if k in wr:
            e["write_kb"] = wr[k]
        if k in fe and k in wr:
            e["hbm_bytes_per_launch"] = (2 * fe[k] + wr[k]) * 1024
            e["hbm_bytes_per_launch_raw"] = (fe[k] + wr[k]) * 1024
        if k in va:
            e["valu_insts_per_launch"] = va[k]
            if k in st and st[k]["avg_ns"] > 0:  # wave instructions x 64 lanes / time / peak
                e["valu_frac"] = va[k] * 64 / st[k]["avg_ns"] / VALU_PEAK_OPS_PER_NS
        if k in fe_mx and k in wr_mx:  # the largest dispatch (its duration: the kernel's MaxNs)
            e["largest"] = {"hbm_bytes": (2 * fe_mx[k] + wr_mx[k]) * 1024, "fetch_kb_raw": fe_mx[k],
                            "write_kb": wr_mx[k]}
            if k in va_mx and k in st and st[k].get("max_ns"):
                e["largest"]["valu_frac"] = va_mx[k] * 64 / st[k]["max_ns"] / VALU_PEAK_OPS_PER_NS
                e["largest"]["ns"] = st[k]["max_ns"]
        out[k] = e
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
