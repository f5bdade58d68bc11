"""Summarise rocprofv3 --pmc runs: per logical HIP op (bench.py's spmm_fwd / spmm_bwd = main +
chunk + tree + fixup kernels of one launch) the HBM bytes per launch, calibrated on the copy
kernel of tools/pmc_calib.py.  usage: pmc_summary.py FETCH_DIR WRITE_DIR CAL_FETCH_DIR
CAL_WRITE_DIR OUT_JSON N E"""
import csv
import glob
import json
import sys
from collections import defaultdict


def load(d):
    f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
    rows = list(csv.DictReader(open(f[0])))
    out = defaultdict(list)   # kernel name -> list of values (per dispatch)
    for r in rows:
        out[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return out


def group(name):
    """logical op of a kernel: spmm_main / spmm_chunks / spmm_fixup<T, LPR, NV, MODE, ...> with
    MODE 0 = forward, 1..4 = backward variants (re_spmm.hip); the shared partial-sum tree; the
    fused output head."""
    if "regnn::" not in name:
        return None
    if "head_fwd_kernel" in name:
        return "head_fwd"
    for k in ("spmm_main", "spmm_chunks", "spmm_fixup"):
        if k in name:
            targs = name[name.index("<") + 1:name.index(">")].split(",")
            return "spmm_fwd" if int(targs[3]) == 0 else "spmm_bwd"
    if "partial_reduce" in name:
        return "spmm_tree"
    return None


def main():
    fd, wd, cfd, cwd, out_json, N, E = sys.argv[1:8]
    fetch, write = load(fd), load(wd)
    cal_f = max(sum(v) for k, v in load(cfd).items() if "regnn" not in k) * 1024
    cal_w = max(sum(v) for k, v in load(cwd).items() if "regnn" not in k) * 1024
    true_bytes = 4 * (1 << 30)
    f_scale, w_scale = true_bytes / cal_f, true_bytes / cal_w
    res = {}
    for op in ("spmm_fwd", "spmm_bwd", "head_fwd"):
        fk = {k: v for k, v in fetch.items() if group(k) == op}
        if not fk:
            continue
        wk = {k: v for k, v in write.items() if group(k) == op}
        launches = max(len(v) for v in fk.values())
        # tree kernels are shared by fwd/bwd; split them evenly per launch (small)
        spmm = op.startswith("spmm")
        tf = sum(sum(v) for k, v in fetch.items() if group(k) == "spmm_tree") if spmm else 0
        tw = sum(sum(v) for k, v in write.items() if group(k) == "spmm_tree") if spmm else 0
        fb = (sum(sum(v) for v in fk.values()) + tf / 2) * 1024 / launches
        wb = (sum(sum(v) for v in wk.values()) + tw / 2) * 1024 / launches
        res[op] = {"fetch_bytes_raw": fb, "write_bytes_raw": wb,
                   "fetch_scale": f_scale, "write_scale": w_scale,
                   "bytes_per_launch": fb * f_scale + wb * w_scale, "launches": launches,
                   "kernels": sorted(fk)}
    res["calibration"] = {"copy_bytes": true_bytes, "FETCH_SIZE_bytes": cal_f,
                          "WRITE_SIZE_bytes": cal_w}
    res["graph"] = {"N": int(N), "E": int(E)}
    json.dump(res, open(out_json, "w"), indent=1)
    for op in [o for o in ("spmm_fwd", "spmm_bwd", "head_fwd") if o in res]:
        with open(out_json.replace("pmc_mag.json", f"pmc_mag_{op}.json"), "w") as f:
            json.dump(res[op] | {"calibration": res["calibration"]}, f, indent=1)
    print(json.dumps({k: v.get("bytes_per_launch") if isinstance(v, dict) else v
                      for k, v in res.items()}, indent=1))


if __name__ == "__main__":
    main()
