"""Turn rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs) into the
per-step HBM traffic of one mode of bench.py, corrected as
MI355X_MICROARCH.md §HBM prescribes (FETCH_SIZE reads 1/2 of wide coalesced
streaming reads on gfx950 -> x2; WRITE_SIZE exact for 16-B stores; values in
KiB).  The x2 is calibrated for 16-B/lane streams only: tools/probes/
fetch_probe.hip measures the factor for this kernel's access widths.

mode "ref":   g2k_scene_kernel<..., false> (g2k_step_fused_f32)
mode "train": g2k_scene_kernel<..., true> + g2k_grad_rows_kernel + g2k_update_kernel
              (one g2k_train_step_f32)

usage: collect_pmc.py FETCH_DIR WRITE_DIR CONFIG OUT_JSON MODE"""
import collections, csv, glob, json, os, re, sys

SCENE = re.compile(r"g2k_scene_kernel<\s*\d+,\s*\d+,\s*(true|false)")


def kernel_of(name, mode):
    """The bench kernel a trace row belongs to in this mode, or None: the
    scene kernel's third template argument is GRAD (false: reference mode)."""
    m = SCENE.search(name)
    if m:
        return "g2k_scene_kernel" if (m.group(1) == "true") == (mode == "train") else None
    if mode == "train":
        for k in ("g2k_grad_rows_kernel", "g2k_update_kernel"):
            if k in name:
                return k
    return None


def per_kernel(d, counter, mode):
    vals = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            k = kernel_of(r["Kernel_Name"], mode)
            if k:
                vals[k].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items() if v}


sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodaltraj_2_amd.build import kernel_tree_sha  # noqa: E402

mode = sys.argv[5] if len(sys.argv) > 5 else "ref"
fetch = per_kernel(sys.argv[1], "FETCH_SIZE", mode)
write = per_kernel(sys.argv[2], "WRITE_SIZE", mode)
kib = 1024.0
raw_f = sum(fetch.values()) * kib
raw_w = sum(write.values()) * kib
res = {"config": sys.argv[3], "mode": mode,
       "fetch_size_bytes_raw": raw_f, "write_size_bytes": raw_w,
       "hbm_bytes_per_launch": 2 * raw_f + raw_w,
       "correction": "FETCH_SIZE x2 (gfx950 reports half of wide coalesced reads), WRITE_SIZE as is",
       "per_kernel_kib": {"FETCH_SIZE": fetch, "WRITE_SIZE": write},
       "kernel_tree_sha": kernel_tree_sha()}
json.dump(res, open(sys.argv[4], "w"), indent=1)
print(json.dumps(res))
