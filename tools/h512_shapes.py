"""The GEMM-like ops (and copies) of one eager h512 module-path NS step with their shapes and
device times (torch.profiler, record_shapes): which products still go to hipBLASLt and why.
usage on the GPU box: python tools/h512_shapes.py [--scale 1.0]"""
import argparse
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "re-gnn_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=1.0)
    a = ap.parse_args()
    import bench
    args = argparse.Namespace(scale=a.scale, zipf=0.0, hidden=512, dropout=0.5, batch=512)
    tr, _ = bench.build_ns(args, "cuda")
    for _ in range(3):
        tr.step()
    torch.cuda.synchronize()
    from torch.profiler import profile, ProfilerActivity
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as p:
        tr.step()
        torch.cuda.synchronize()
    agg = defaultdict(lambda: [0, 0.0])
    for e in p.key_averages(group_by_input_shape=True):
        if any(k in e.key for k in ("mm", "linear", "copy", "matmul", "cat", "foreach")):
            dt = getattr(e, "device_time_total", None) or getattr(e, "cuda_time_total", 0)
            agg[(e.key, str(e.input_shapes)[:120])][0] += e.count
            agg[(e.key, str(e.input_shapes)[:120])][1] += dt
    for (k, s), (c, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:40]:
        print(f"{t:10.1f} us  x{c:3d}  {k:32s} {s}")


if __name__ == "__main__":
    main()
