"""Per-phase dispatch durations of one kernel in a rocprofv3 kernel trace of
bench.py: dispatches are grouped into runs separated by > 200 us of idle
time, so the timed steps (launches overlapping on several streams / hardware
queues) and the roofline's pass (launches back to back on one stream, what
bench.py's kernel_us measures with HIP events) are reported apart.
    python tools/trace_split.py TRACE_DIR [KERNEL_SUBSTRING]"""
import csv
import glob
import os
import statistics
import sys

d = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "g2k_scene_kernel<2, 4, false"
f = sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True))[0]
rows = sorted((r for r in csv.DictReader(open(f)) if pat in r["Kernel_Name"]),
              key=lambda r: int(r["Start_Timestamp"]))
runs = []
for i, r in enumerate(rows):
    if i == 0 or int(r["Start_Timestamp"]) - int(rows[i - 1]["End_Timestamp"]) > 200_000:
        runs.append([])
    runs[-1].append(r)
print(f"{pat}: {len(rows)} dispatches in {len(runs)} runs ({os.path.relpath(f)})")
for k, run in enumerate(runs):
    us = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in run]
    span = (int(run[-1]["End_Timestamp"]) - int(run[0]["Start_Timestamp"])) / 1e3
    queues = len({r["Queue_Id"] for r in run})
    print(f"run {k}: {len(run)} dispatches on {queues} hardware queue(s), per dispatch mean "
          f"{statistics.mean(us):.2f} us (median {statistics.median(us):.2f}, min {min(us):.2f}, "
          f"max {max(us):.2f}); span {span:.1f} us = {span / len(run):.2f} us per dispatch")
