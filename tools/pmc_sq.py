"""Summarise rocprofv3 --pmc passes (any counters) per kernel: mean counter
value per dispatch for every kernel whose name contains 'g2k_'.

usage: pmc_sq.py DIR [DIR ...]"""
import collections, csv, glob, os, sys

vals = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "g2k_" not in k:
                continue
            k = k.split("g2k_", 1)[1].split("(")[0].split("<")[0]
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in vals.items():
    print(f"== g2k_{k}")
    for c in sorted(cs):
        v = cs[c]
        print(f"  {c:32s} {sum(v) / len(v):16.1f}   (n={len(v)})")
