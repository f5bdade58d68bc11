"""Phase timestamps of the two-layer NS step's kernels (an instrumented library build:
-DREGNN_NSM2_PHASES, loaded through REGNN_LIB). usage on the GPU box:
    REGNN_LIB=$PWD/ab/libregnn_phases.so python tools/nsm2_phases.py [--pipeline]
Prints, for the last of a few eager steps, each marked point of agg0 / head / bwd0 / finalize as
microseconds after agg0's first block started (mean and max over blocks 0..31)."""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "re-gnn_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pipeline", action="store_true")
    ap.add_argument("--scale", type=float, default=10.0)
    a = ap.parse_args()
    import bench
    from regnn_hip import _lib as L
    args = argparse.Namespace(scale=a.scale, zipf=1.1, hidden=64, dropout=0.5, batch=512)
    tr, info = bench.build_ns(args, torch.device("cuda", 0))
    if not a.pipeline:
        tr.pipelined = False
    f = L._so.regnn_nsm2_phases
    f.argtypes = [ctypes.c_void_p]
    buf = np.zeros((4, 32, 16), np.uint64)
    fe = L._so.regnn_nsm2_edges
    fe.argtypes = [ctypes.c_void_p]
    edges = np.zeros((5, 2, 4096), np.uint64)
    for i in range(8):
        if i == 7:
            L._so.regnn_nsm2_edges_reset()
        tr.step()
        torch.cuda.synchronize()
    f(buf.ctypes.data)
    fe(edges.ctypes.data)
    s = tr.sampler
    if s.csc[0] is not None:
        _, cptr, _, clong = s.csc[0]
        nl = int(clong[0])
        ids = clong[1:1 + nl].long()
        m = (cptr[ids + 1] - cptr[ids]).cpu().numpy()
        print(f"hop-0 block: {int(s.sizes[1])} sources, {int(s.sizes[8])} edges; {nl} hub rows, "
              f"entries max {m.max() if nl else 0} p50 {np.median(m) if nl else 0} sum {m.sum()}; "
              f"pieces {int(clong[1929])}")
    e0 = edges[0, 0][edges[0, 0] > 0]
    t0 = int(e0.min()) if e0.size else int(buf[0, :, 0][buf[0, :, 0] > 0].min())
    names = {0: "agg0", 1: "head", 2: "bwd0/gath", 3: "finalize"}
    if hasattr(L._so, "regnn_nsm2_gpieces"):
        gp = np.zeros((64, 8), np.uint64)
        L._so.regnn_nsm2_gpieces.argtypes = [ctypes.c_void_p]
        L._so.regnn_nsm2_gpieces(gp.ctypes.data)
        for j in range(64):
            row = gp[j].astype(np.int64)
            if row[0] <= 0:
                continue
            marks = " ".join(f"{(x - t0) / 100.0:7.2f}" for x in row[:4] if x > 0)
            print(f"piece {j:2d}: {marks}")
    for k, nm in enumerate(["agg0", "head", "gather", "bwd0", "finalize"]):
        en, ex = edges[k, 0].astype(np.int64), edges[k, 1].astype(np.int64)
        ok = (en > 0) & (ex > 0)
        if not ok.any():
            continue
        en, ex = (en[ok] - t0) / 100.0, (ex[ok] - t0) / 100.0
        dur = ex - en
        print(f"{nm:9s} blocks {ok.sum():5d}: entry {en.min():7.2f}..{en.max():7.2f}  exit "
              f"{ex.min():7.2f}..{ex.max():7.2f} (p50 {np.percentile(ex, 50):7.2f} p90 "
              f"{np.percentile(ex, 90):7.2f})  dur p50 {np.percentile(dur, 50):6.2f} max "
              f"{dur.max():6.2f}  slowest block {int(np.nonzero(ok)[0][np.argmax(dur)])}")
    for k in range(4):
        for p in range(16):
            col = buf[k, :, p].astype(np.int64)
            if not (col > 0).any():
                continue
            us = (col[col > 0] - t0) / 100.0          # wall_clock64: 100 MHz
            print(f"{names[k]:9s} mark {p:2d}: mean {us.mean():8.2f} us  min {us.min():8.2f}  "
                  f"max {us.max():8.2f}  (blocks {int((col > 0).sum())})")


if __name__ == "__main__":
    main()
