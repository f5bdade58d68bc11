"""Interleaved A/B of SpMM launch configurations in ONE process (cdna guide §5.4 rule 24).

    python tools/ab_spmm.py [--scale 10] [--rounds 5] [--F 64] [--dtype fp32]

Variants cap:split:chunk[:un[:prescale[:rs]]]: grid cap (regnn_tune key 1) x long-segment
split/chunk x rows in flight (key 2) x ops.PRESCALE mode (on/off/auto). Reports per variant the median
ms of spmm_fwd / spmm_bwd (HIP events on the launch stream) and GB/s on SURVEY §8d bytes.
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "re-gnn_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=10.0)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--F", type=int, default=64)
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("--dropout", type=float, default=0.0, help="fused dropout of the gathered rows")
    ap.add_argument("--variants", default="res:256:256,cap2048:256:256,res:1024:256,res:256:512")
    args = ap.parse_args()
    from regnn_hip import _lib as L, ops, profile, synth
    from regnn_hip.graph import RelGraph
    dev = torch.device("cuda")
    gd = synth.mag_like(args.scale, seed=0, device=dev)
    e_feat = gd["rel"].to(torch.int64)
    dt = torch.float32 if args.dtype == "fp32" else torch.bfloat16
    s = 4 if dt == torch.float32 else 2
    x0 = torch.randn(gd["N"], args.F, device=dev).to(dt)
    gy = torch.randn(gd["N"], args.F, device=dev).to(dt)
    graphs = {}
    variants = []
    for v in args.variants.split(","):
        parts = v.split(":")
        cap, split, chunk = parts[:3]
        un = int(parts[3]) if len(parts) > 3 else 0
        pre = parts[4] if len(parts) > 4 else "auto"       # ops.PRESCALE mode
        rs = int(parts[5]) if len(parts) > 5 else 0        # regnn_row_scale rows in flight (key 4)
        key = (int(split), int(chunk))
        if key not in graphs:
            graphs[key] = RelGraph(gd["src"], gd["dst"], gd["N"], dev, split=key[0], chunk=key[1])
        variants.append((v, 0 if cap == "res" else int(cap[3:]), graphs[key], un, pre, rs))
    E, N = graphs[next(iter(graphs))].E, gd["N"]
    F = args.F
    fwd_b = E * (F * s + 9) + N * (F * s + 8)
    bwd_b = E * (F * s + 9) + N * (3 * F * s + 12)
    res = {v[0]: {"fwd": [], "bwd": []} for v in variants}
    for r in range(args.rounds + 1):
        for name, cap, rg, un, pre, rs in variants:
            ops.PRESCALE["mode"] = ops.PRESCALE["bwd"] = pre
            L._so.regnn_tune(4, rs)
            L._so.regnn_tune(1, cap)
            L._so.regnn_tune(2, un)
            pack = rg.rel_pack(e_feat, 11)
            tab = torch.full((11, 1), 0.9, device=dev, requires_grad=True)
            x = x0.clone().requires_grad_(True)
            profile.enable(True)
            norm = ops.degree_norm(rg, pack, tab)
            y = ops.re_spmm(rg, x, tab, pack, pre=norm, post=norm, dropout=args.dropout)
            y.backward(gy)
            torch.cuda.synchronize()
            st = profile.summary()
            profile.enable(False)
            if r > 0:   # round 0 = warm-up
                res[name]["fwd"].append(st["spmm_fwd"][1])
                res[name]["bwd"].append(st["spmm_bwd"][1])
            del x, y, norm
    L._so.regnn_tune(1, 0)
    L._so.regnn_tune(2, 0)
    L._so.regnn_tune(4, 0)
    out = {}
    for name, d in res.items():
        f, b = statistics.median(d["fwd"]), statistics.median(d["bwd"])
        out[name] = {"fwd_ms": round(f, 3), "bwd_ms": round(b, 3),
                     "fwd_TBs": round(fwd_b / f / 1e9, 3), "bwd_TBs": round(bwd_b / b / 1e9, 3),
                     "fwd_min": round(min(d["fwd"]), 3), "bwd_min": round(min(d["bwd"]), 3)}
    print(json.dumps({"scale": args.scale, "F": F, "dtype": args.dtype, "dropout": args.dropout, "E": E, "N": N,
                      "variants": out}, indent=1))


if __name__ == "__main__":
    main()
