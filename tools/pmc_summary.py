"""Summarise rocprofv3 --pmc runs: per logical HIP op (bench.py's spmm_fwd / spmm_bwd = main +
chunk + tree + fixup kernels of one launch) the HBM bytes per launch, calibrated on the copy
kernel of tools/pmc_calib.py.  usage: pmc_summary.py FETCH_DIR WRITE_DIR CAL_FETCH_DIR
CAL_WRITE_DIR OUT_JSON N E [DTYPE]

Dispatches are attributed in dispatch order: a row_scale pass (the pre-scale of regnn_row_scale)
belongs to the SpMM op whose main kernel follows it, the partial-sum tree and fixup kernels to the
op whose main kernel precedes them."""
import csv
import glob
import json
import sys
from collections import defaultdict


def load(d):
    """-> list of (dispatch id, kernel name, value) in dispatch order."""
    f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
    rows = list(csv.DictReader(open(f[0])))
    out = [(int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"])) for r in rows]
    return sorted(out)


def kind(name):
    if "regnn::" not in name:
        return None
    if "head_fwd_kernel" in name or "head_fwd_x6_kernel" in name:
        return "head_fwd"
    if "spmm_main" in name:
        targs = name[name.index("<") + 1:name.index(">")].split(",")
        return "spmm_fwd" if int(targs[3]) == 0 else "spmm_bwd"
    if "row_scale" in name:
        return "pre"
    if "spmm_chunks" in name or "spmm_fixup" in name or "partial_reduce" in name:
        return "post"
    return None


def per_op(disp):
    """op -> (summed counter value, kernel names, launches of its main kernel)."""
    tot, names, launches = defaultdict(float), defaultdict(set), defaultdict(int)
    pending, pend_names, cur = 0.0, set(), None
    for _, name, v in disp:
        k = kind(name)
        if k == "pre":
            pending += v
            pend_names.add(name)
        elif k in ("spmm_fwd", "spmm_bwd"):
            cur = k
            tot[k] += v + pending
            names[k] |= pend_names | {name}
            launches[k] += 1
            pending, pend_names = 0.0, set()
        elif k == "post" and cur is not None:
            tot[cur] += v
            names[cur].add(name)
        elif k == "head_fwd":
            cur = None
            tot[k] += v
            names[k].add(name)
            launches[k] += 1
        elif k is None and "regnn::" in name:
            cur = None
    return tot, names, launches


def main():
    fd, wd, cfd, cwd, out_json, N, E = sys.argv[1:8]
    dtype = sys.argv[8] if len(sys.argv) > 8 else "fp32"
    (fetch, fnames, flaunch), (write, _, _) = per_op(load(fd)), per_op(load(wd))
    cal_f = max(v for _, k, v in load(cfd) if "regnn" not in k) * 1024
    cal_w = max(v for _, k, v in load(cwd) if "regnn" not in k) * 1024
    true_bytes = 4 * (1 << 30)
    f_scale, w_scale = true_bytes / cal_f, true_bytes / cal_w
    res = {}
    for op in ("spmm_fwd", "spmm_bwd", "head_fwd"):
        if not flaunch.get(op):
            continue
        launches = flaunch[op]
        fb = fetch[op] * 1024 / launches
        wb = write[op] * 1024 / launches
        res[op] = {"fetch_bytes_raw": fb, "write_bytes_raw": wb,
                   "fetch_scale": f_scale, "write_scale": w_scale,
                   "bytes_per_launch": fb * f_scale + wb * w_scale, "launches": launches,
                   "kernels": sorted(fnames[op])}
    res["calibration"] = {"copy_bytes": true_bytes, "FETCH_SIZE_bytes": cal_f,
                          "WRITE_SIZE_bytes": cal_w}
    res["graph"] = {"N": int(N), "E": int(E)}
    res["dtype"] = dtype
    # the kernel code the counters were collected on (bench.py refuses a stale summary)
    sys.path.insert(0, __file__.rsplit("/tools/", 1)[0] + "/re-gnn_amd")
    from regnn_hip.build import kernel_hash
    res["code_hash"] = kernel_hash()
    json.dump(res, open(out_json, "w"), indent=1)
    print(json.dumps({k: v.get("bytes_per_launch") if isinstance(v, dict) and "fetch_scale" in v
                      else v for k, v in res.items()}, indent=1))


if __name__ == "__main__":
    main()
