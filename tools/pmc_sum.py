"""Summarize tools/ab_pmc.sh output: python tools/pmc_sum.py gpurun_out/TAG"""
import csv, collections, glob, os, sys
base = sys.argv[1]
names = sorted({os.path.basename(d).rsplit("_p", 1)[0] for d in glob.glob(base + "/*_p*") if os.path.isdir(d)})
rows = collections.OrderedDict()
for n in names:
    agg = collections.defaultdict(list)
    for p in glob.glob(f"{base}/{n}_p*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    rows[n] = {k: sum(v) / len(v) for k, v in agg.items()}
keys = sorted({k for r in rows.values() for k in r})
print("%-22s" % "counter" + "".join("%14s" % n for n in rows))
for k in keys:
    print("%-22s" % k + "".join("%14.4g" % rows[n].get(k, float("nan")) for n in rows))
