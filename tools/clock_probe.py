"""Probe: does a GPU that was idle before a timed region run slower for its first milliseconds?
Times two fixed workloads (20 4096^3 fp32 GEMMs; 400 small elementwise launches) after: a busy
GPU (work in flight, no sync), a sync (~0.1 ms idle) and a 20 ms sleep."""
import statistics
import time

import torch


def main():
    dev = torch.device("cuda", 0)
    A = torch.randn(4096, 4096, device=dev)
    x = torch.randn(4 << 20, device=dev)
    s = torch.cuda.current_stream()

    def gemms():
        for _ in range(20):
            A.mm(A)

    def small():
        for _ in range(400):
            x.mul_(1.0000001)

    for _ in range(3):
        gemms(); small()
    torch.cuda.synchronize()
    for name, work in (("gemm x20", gemms), ("small x400", small)):
        for pre in ("busy", "sync", "sleep20ms"):
            ts = []
            for _ in range(7):
                torch.cuda.synchronize()
                if pre == "busy":
                    gemms()
                elif pre == "sleep20ms":
                    time.sleep(0.02)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                work()
                e1.record(s)
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            print(f"{name:11s} pre={pre:9s} median {statistics.median(ts):7.3f} ms  "
                  f"min {min(ts):7.3f} ms", flush=True)


if __name__ == "__main__":
    main()
