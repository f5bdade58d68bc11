"""A/B timing of the dense weight-gradient forms at mag-10x shapes (GPU)."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "re-gnn_amd"))
import torch
from regnn_hip import ops


def t(fn, it=10):
    fn(); torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / it


for rows, k, m in ((7_363_890, 128, 64), (11_346_490, 128, 64), (7_363_890, 64, 349)):
    x = torch.randn(rows, k, device="cuda")
    g = torch.randn(rows, m, device="cuda")
    res = {"mm": t(lambda: g.t() @ x)}
    for c in (4096, 16384, 32768, 131072):
        res[f"bmm{c}"] = t(lambda: ops.batched_wgrad(g, x, chunk=c))
    ref = g.t() @ x
    err = (ops.batched_wgrad(g, x) - ref).abs().max().item() / ref.abs().max().item()
    gb = rows * (k + m) * 4 / 1e9
    print(rows, k, m, {a: f"{v:.2f}ms {gb / v:.2f}TB/s" for a, v in res.items()}, f"err {err:.1e}",
          flush=True)
    del x, g
