"""A/B timing of the fused output head (regnn_head_fwd variants, tune key 3) against
hipBLASLt addmm + regnn_softmax_xent, at the mag-10x shape (GPU)."""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "re-gnn_amd"))
import torch
from regnn_hip import _lib as L

N, n, K = int(sys.argv[1]) if len(sys.argv) > 1 else 19_397_430, 7_363_890, 64
C = int(os.environ.get("HEAD_C", "349"))
h = torch.randn(N, K, device="cuda")
W = torch.randn(C, K, device="cuda") * 0.1
b = torch.randn(C, device="cuda") * 0.1
y = torch.randint(0, C, (n,), device="cuda")
LD = int(os.environ.get("HEAD_LD", str(16 * ((C + 15) // 16))))   # row stride of logits / p
logits = torch.empty(N, LD, device="cuda")
p = torch.empty(n, LD, device="cuda")
lr = torch.empty(n, device="cuda")


def fused():
    L.call("regnn_head_fwd", L.ptr(h), N, K, L.ptr(W), L.ptr(b), C, LD, L.ptr(y), n, 1.0 / n,
           L.ptr(logits), L.ptr(p), L.ptr(lr), L.stream())


def unfused():
    z = torch.addmm(b, h, W.t())
    L.call("regnn_softmax_xent", L.ptr(z), n, C, C, L.ptr(y), 1.0 / n, L.ptr(p[:, :C].contiguous()), L.ptr(lr),
           L.stream())


def t(fn, it=5):
    fn(); torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / it


res = {}
outs = {}
VARIANTS = [int(v) for v in os.environ.get("HEAD_VARIANTS", "0,1,2,4").split(",")]
for v in VARIANTS:
    L._so.regnn_tune(3, v)
    res[f"fused_v{v}"] = t(fused)
    if v not in (2, 4):
        outs[v] = (logits.clone(), p.clone())
L._so.regnn_tune(3, 0)
res["addmm+xent"] = t(unfused)
same = {v: all(torch.equal(outs[VARIANTS[0]][i], o[i]) for i in range(2)) for v, o in outs.items()}
print('variants: 1 no-prefetch, 2 no logits store, 4 no loss epilogue')
gb = (N * K + N * C + n * C) * 4 / 1e9
tf = 2 * N * C * K / 1e12
print({k: f"{v:.2f}ms {gb / v:.2f}TB/s {tf / v * 1e3:.0f}TF" for k, v in res.items()},
      "variants bit-identical:", same, flush=True)
