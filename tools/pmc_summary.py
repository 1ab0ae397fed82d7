"""Summarise a rocprofv3 --pmc / --kernel-trace CSV directory per kernel."""
import collections, csv, glob, os, sys

d = sys.argv[1]
for f in sorted(glob.glob(os.path.join(d, "*counter_collection.csv"))):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"][:70]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, dd in agg.items():
        print("PMC", k, {c: round(sum(v) / len(v)) for c, v in dd.items()})
for f in sorted(glob.glob(os.path.join(d, "*kernel_stats.csv"))):
    for r in csv.DictReader(open(f)):
        print("STAT", r["Name"][:70], r["Calls"], r["AverageNs"], r["MinNs"], r["MaxNs"])
