import csv,sys,collections,glob
for f in sorted(glob.glob(sys.argv[1] + '/*/*counter_collection.csv')):
    rows=list(csv.DictReader(open(f)))
    agg=collections.defaultdict(list)
    for r in rows: agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(f)
    for k,v in agg.items(): print(' ', k, len(v), sum(v)/len(v))
