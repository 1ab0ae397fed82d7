"""Span of the timed graph replay in a rocprofv3 kernel trace of bench.py
(development tool): per-dispatch start / end of the g2k_scene_kernel
forward launches, grouped into replays by gaps, and for the last replay of
`--steps` launches: first start -> last end, the fill (first end - first
start) and drain, and the steady spacing of launch ends.

usage: python tools/trace_span.py TRACE_DIR STEPS"""
import csv
import glob
import os
import sys

d, steps = sys.argv[1], int(sys.argv[2])
rows = []
for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if "g2k_scene_kernel" in r["Kernel_Name"] and "true" not in r["Kernel_Name"].split("<")[1].split(",")[2]:
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]))
rows.sort()
print("forward scene-kernel dispatches:", len(rows))
# replays: the timed one is the last block of `steps` dispatches before the train kernels
starts = [r[0] for r in rows]
ends = [r[1] for r in rows]
# split into groups where the gap between consecutive starts > 50 us
groups, cur = [], [rows[0]]
for a, b in zip(rows, rows[1:]):
    if b[0] - a[0] > 50_000:
        groups.append(cur)
        cur = []
    cur.append(b)
groups.append(cur)
for g in groups:
    s0 = g[0][0]
    e = sorted(x[1] for x in g)
    dur = [(x[1] - x[0]) / 1e3 for x in g]
    print(f"group of {len(g):4d}: span {(max(x[1] for x in g) - s0) / 1e3:8.2f} us  first end {(e[0] - s0) / 1e3:6.2f}  "
          f"per-launch span {(max(x[1] for x in g) - s0) / 1e3 / len(g):6.2f}  mean dur {sum(dur) / len(dur):6.2f}  "
          f"ends steady spacing {((e[-1] - e[len(e) // 4]) / max(1, len(e) - 1 - len(e) // 4)) / 1e3:6.2f}")
