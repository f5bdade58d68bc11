"""Summarise rocprofv3 --pmc runs of the NS bench (bench.py --workload ns): the HBM bytes of one
fused model step (every regnn::nsm:: kernel but Adam, i.e. what bench.py times as `nsm_step`),
per step, calibrated on the copy kernel of tools/pmc_calib.py.

usage: pmc_ns_summary.py FETCH_DIR WRITE_DIR CAL_FETCH_DIR CAL_WRITE_DIR OUT_JSON SCALE BATCH DROPOUT

A step is anchored on its agg0 dispatch (the first model kernel of regnn_nsm_step); the per-step
figure is the counted bytes over the anchored steps / their number."""
import csv
import glob
import json
import sys
from collections import defaultdict


def load(d):
    f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
    rows = list(csv.DictReader(open(f[0])))
    return sorted((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"])) for r in rows)


def model_kernel(name):
    return "regnn::nsm" in name and "adam_flat" not in name      # nsm:: and nsm2:: kernels


def per_step(disp):
    tot, per_k = 0.0, defaultdict(float)
    steps = sum(1 for _, n, _ in disp if "regnn::nsm" in n and "agg0" in n and "kernel" in n)
    for _, n, v in disp:
        if model_kernel(n):
            tot += v
            short = n.split("(")[0].replace("void ", "").replace("regnn::", "")
            per_k[short] += v
    return tot, per_k, steps


def main():
    fd, wd, cfd, cwd, out_json, scale, batch, dropout = sys.argv[1:9]
    ft, fk, fs = per_step(load(fd))
    wt, wk, ws = per_step(load(wd))
    if not fs or fs != ws:
        raise SystemExit(f"step count mismatch / zero: fetch {fs}, write {ws}")
    cal_f = max(v for _, k, v in load(cfd) if "regnn" not in k) * 1024
    cal_w = max(v for _, k, v in load(cwd) if "regnn" not in k) * 1024
    true_bytes = 4 * (1 << 30)
    f_scale, w_scale = true_bytes / cal_f, true_bytes / cal_w
    res = {"nsm_step": {
        "bytes_per_launch": (ft * 1024 * f_scale + wt * 1024 * w_scale) / fs,
        "fetch_bytes_per_launch": ft * 1024 * f_scale / fs,
        "write_bytes_per_launch": wt * 1024 * w_scale / fs,
        "steps": fs,
        "per_kernel_bytes": {k: (fk[k] * 1024 * f_scale + wk.get(k, 0.0) * 1024 * w_scale) / fs
                             for k in sorted(fk)}}}
    # the sampler's outer-hop sums launch (regnn_ns_hop_typed_sums), per dispatch
    def sums(path, scale_):
        v = [x for _, n, x in load(path) if "ns_sample_sums_kernel" in n]
        return (sum(v) * 1024 * scale_ / len(v), len(v)) if v else (None, 0)
    sf, sn = sums(fd, f_scale)
    sw, _ = sums(wd, w_scale)
    if sn:
        res["ns_sums"] = {"bytes_per_launch": sf + sw, "fetch_bytes_per_launch": sf,
                          "write_bytes_per_launch": sw, "launches": sn}
    res["calibration"] = {"copy_bytes": true_bytes, "FETCH_SIZE_bytes": cal_f,
                          "WRITE_SIZE_bytes": cal_w}
    res["config"] = {"scale": float(scale), "batch": int(batch), "fanout": [25, 20],
                     "hidden": 64, "dropout": float(dropout)}
    sys.path.insert(0, __file__.rsplit("/tools/", 1)[0] + "/re-gnn_amd")
    from regnn_hip.build import NS_PMC_SOURCES, kernel_hash
    res["code_hash"] = kernel_hash(NS_PMC_SOURCES)
    from regnn_hip.build import NS_SUMS_SOURCES
    res["sums_code_hash"] = kernel_hash(NS_SUMS_SOURCES)
    json.dump(res, open(out_json, "w"), indent=1)
    print(json.dumps(res["nsm_step"], indent=1))


if __name__ == "__main__":
    main()
