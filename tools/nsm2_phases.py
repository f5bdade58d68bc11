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
    for i in range(8):
        tr.step()
        torch.cuda.synchronize()
    f(buf.ctypes.data)
    t0 = int(buf[0, :, 0][buf[0, :, 0] > 0].min())
    names = {0: "agg0", 1: "head", 2: "bwd0", 3: "finalize"}
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
