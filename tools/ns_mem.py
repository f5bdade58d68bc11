"""HBM the NS bench trainer holds at a given sampling lookahead (REGNN_NS_AHEAD), after capture."""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "re-gnn_amd"))
sys.path.insert(0, ROOT)


def main():
    import bench
    args = argparse.Namespace(scale=10.0, zipf=1.1, hidden=64, dropout=0.5, batch=512)
    dev = torch.device("cuda", 0)
    tr, info = bench.build_ns(args, dev)
    torch.cuda.synchronize()
    base = torch.cuda.memory_allocated(dev)
    import time
    t0 = time.perf_counter()
    tr.capture(warmup=2)
    torch.cuda.synchronize()
    tc = time.perf_counter() - t0
    tr.run_steps(16)
    torch.cuda.synchronize()
    print(f"ahead {tr.ahead}: slots {len(tr.slots)}, allocated {base / 2**30:.2f} GiB at build, "
          f"{torch.cuda.memory_allocated(dev) / 2**30:.2f} GiB after capture, peak "
          f"{torch.cuda.max_memory_allocated(dev) / 2**30:.2f} GiB; capture {tc:.2f} s "
          f"({len(tr.graph_groups)} multi-step graphs)")


if __name__ == "__main__":
    main()
