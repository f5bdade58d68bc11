"""Per-kernel HBM bytes per dispatch from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs (separate
passes), calibrated on the copy kernel of tools/pmc_calib.py (gfx950: FETCH_SIZE reads back half
the bytes a copy reads, WRITE_SIZE exact), next to each kernel's mean duration from a
--kernel-trace --stats run of the same command.

usage: pmc_kernels.py FETCH_DIR WRITE_DIR CAL_FETCH_DIR CAL_WRITE_DIR STATS_CSV OUT_JSON MATCH...
Only kernels whose name contains one of MATCH are summarised."""
import csv
import glob
import json
import sys
from collections import defaultdict


def load(d):
    f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
    return [(r["Kernel_Name"], float(r["Counter_Value"])) for r in csv.DictReader(open(f[0]))]


def short(name):
    return name.split("(")[0].replace("void ", "")


def main():
    fd, wd, cfd, cwd, stats, out, *match = sys.argv[1:]
    true_bytes = 4 * (1 << 30)
    f_scale = true_bytes / (max(v for k, v in load(cfd) if "regnn" not in k) * 1024)
    w_scale = true_bytes / (max(v for k, v in load(cwd) if "regnn" not in k) * 1024)
    acc = defaultdict(lambda: [0.0, 0, 0.0, 0])
    for name, v in load(fd):
        if any(m in name for m in match):
            a = acc[short(name)]
            a[0] += v * 1024 * f_scale
            a[1] += 1
    for name, v in load(wd):
        if any(m in name for m in match):
            a = acc[short(name)]
            a[2] += v * 1024 * w_scale
            a[3] += 1
    dur = {}
    for r in csv.DictReader(open(stats)):
        dur[short(r["Name"])] = float(r["AverageNs"]) / 1e3
    res = {}
    for k, (fb, fn, wb, wn) in sorted(acc.items()):
        if not fn or not wn:
            continue
        b = fb / fn + wb / wn
        us = dur.get(k)
        res[k] = {"bytes_per_dispatch": b, "fetch_bytes": fb / fn, "write_bytes": wb / wn,
                  "dispatches": fn, "mean_us": us,
                  "hbm_tb_s": None if not us else b / (us * 1e-6) / 1e12}
    res["_calibration"] = {"copy_bytes": true_bytes, "fetch_scale": f_scale, "write_scale": w_scale}
    json.dump(res, open(out, "w"), indent=1)
    for k, v in res.items():
        if not k.startswith("_"):
            print(f"{k[:70]:70s} {v['bytes_per_dispatch'] / 1e9:8.3f} GB  {v['mean_us'] or 0:9.1f} us"
                  f"  {v['hbm_tb_s'] or 0:6.2f} TB/s")


if __name__ == "__main__":
    main()
