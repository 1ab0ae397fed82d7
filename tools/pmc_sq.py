"""Summarise rocprofv3 --pmc passes (any counters) per kernel: mean counter
value per dispatch for every kernel whose name contains 'g2k_' (template
arguments kept: the forward and train builds of the scene kernel apart), and
the derived issue fractions when the counters are present.

usage: pmc_sq.py DIR [DIR ...]"""
import collections
import csv
import glob
import os
import sys

vals = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "g2k_" not in k:
                continue
            k = k.split("g2k_", 1)[1].split("(")[0]
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in sorted(vals.items()):
    print(f"== g2k_{k}")
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    for c in sorted(m):
        print(f"  {c:32s} {m[c]:16.1f}   (n={len(cs[c])})")
    wc = m.get("SQ_WAVE_CYCLES")
    if wc:
        for c in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_VALU",
                  "SQ_ACTIVE_INST_LDS"):
            if c in m:
                print(f"  {c + ' / WAVE_CYCLES':45s} {m[c] / wc:8.3f}")
    if "SQ_BUSY_CYCLES" in m and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
        print(f"  {'MFMA busy / (4 SIMD x BUSY_CYCLES)':45s} "
              f"{m['SQ_VALU_MFMA_BUSY_CYCLES'] / (4 * 256 * m['SQ_BUSY_CYCLES'] / 8):8.3f}  (per-CU SIMDs, BUSY summed over 8 XCDs: an estimate)")
