"""Turn rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs) into the
per-launch HBM traffic of one g2k_step_fused_f32 (both kernels), corrected as
MI355X_MICROARCH.md §HBM prescribes (FETCH_SIZE reads 1/2 of wide coalesced
streaming reads on gfx950 -> x2; WRITE_SIZE exact for 16-B stores; values in KiB).

usage: collect_pmc.py FETCH_DIR WRITE_DIR CONFIG OUT_JSON"""
import collections, csv, glob, json, os, sys

KERNELS = ("g2k_scene_kernel", "g2k_frames_kernel", "g2k_recur_kernel")


def per_kernel(d, counter):
    vals = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            for k in KERNELS:
                if k in r["Kernel_Name"]:
                    vals[k].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items() if v}


fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
write = per_kernel(sys.argv[2], "WRITE_SIZE")
kib = 1024.0
raw_f = sum(fetch.values()) * kib
raw_w = sum(write.values()) * kib
res = {"config": sys.argv[3],
       "fetch_size_bytes_raw": raw_f, "write_size_bytes": raw_w,
       "hbm_bytes_per_launch": 2 * raw_f + raw_w,
       "correction": "FETCH_SIZE x2 (gfx950 reports half of wide coalesced reads), WRITE_SIZE as is",
       "per_kernel_kib": {"FETCH_SIZE": fetch, "WRITE_SIZE": write}}
json.dump(res, open(sys.argv[4], "w"), indent=1)
print(json.dumps(res))
