"""Probe: where the fixed cost of a short timed NS run goes (the driver times 20 steps).

Builds the bench's NS trainer, captures, then times run_steps(k) under several preambles and
prints, per run: wall ms, host submit ms (run_steps returning), GPU event ms on the launch stream.
    python tools/ns_k_probe.py [--ahead G]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seq", default="20,20,20,160,20")
    ap.add_argument("--sweep", default="", help="group lengths m: T(m) median/min of 7 runs")
    ap.add_argument("--pre", default="none", help="sweep preambles: none,spin,spin_sync,sleep,self")
    a0 = ap.parse_args()
    args = argparse.Namespace(scale=10.0, zipf=1.1, hidden=64, dropout=0.5, batch=512)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    tr, info = bench.build_ns(args, dev)
    for _ in range(5):
        tr.step()
    tr.capture(warmup=2)
    tr.run_steps(5)
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    if a0.sweep:
        import statistics
        A = torch.randn(4096, 4096, device=dev)

        def spin():                     # ~3 ms of GPU work on the launch stream
            for _ in range(24):
                A.mm(A)
        for m, pre in [(int(x), p) for p in a0.pre.split(",") for x in a0.sweep.split(",")]:
            ts = []
            for _ in range(7):
                torch.cuda.synchronize()
                if pre in ("spin", "spin_sync"):
                    spin()
                if pre == "spin_sync":
                    torch.cuda.synchronize()
                if pre == "sleep":             # 20 ms of GPU idle before the run
                    time.sleep(0.02)
                if pre == "self":               # our own steps in flight (no sync) before it
                    tr.run_steps(16)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                tr.run_steps(m)
                e1.record(s)
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3)
            print(f"m={m:4d} pre={pre:9s} T(m) median {statistics.median(ts):8.1f} us  min {min(ts):8.1f} us  "
                  f"per step {statistics.median(ts) / m:6.1f} us", flush=True)
        return
    for pre in ("edges_total", "none"):
        for k in [int(x) for x in a0.seq.split(",")]:
            if pre == "edges_total":
                torch.cuda.synchronize()
                tr.edges_total()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            e0.record(s)
            tr.run_steps(k)
            t_sub = time.perf_counter() - t0
            e1.record(s)
            torch.cuda.synchronize()
            wall = time.perf_counter() - t0
            print(f"pre={pre:11s} k={k:4d} wall {wall*1e3:8.3f} ms ({wall/k*1e6:6.1f} us/step) "
                  f"submit {t_sub*1e3:7.3f} ms  gpu {e0.elapsed_time(e1):8.3f} ms", flush=True)


if __name__ == "__main__":
    main()
