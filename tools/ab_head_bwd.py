"""A/B timing of the output-head backward at the mag-10x shape (GPU): regnn_head_bwd's gh and
wgrad kernels separately vs the hipBLASLt GEMM + chunked bmm + col_sum path."""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "re-gnn_amd"))
import torch
from regnn_hip import _lib as L, ops

n, K, C = 7_363_890, 64, 349
Cp = 16 * ((C + 15) // 16)
h = torch.randn(n, K, device="cuda")
W = torch.randn(C, K, device="cuda") * 0.1
p = torch.randn(n, C, device="cuda") * 1e-3
gh = torch.empty(n, K, device="cuda")
rows = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
slab = torch.zeros(rows, Cp * K + Cp, device="cuda")


def gh_k():
    L.call("regnn_head_bwd", L.ptr(p), n, C, C, K, L.ptr(W), L.ptr(h), None, L.ptr(gh), n, None,
           rows, L.stream())


def wg_k():
    L.call("regnn_head_bwd", L.ptr(p), n, C, C, K, L.ptr(W), L.ptr(h), None, None, 0, L.ptr(slab),
           rows, L.stream())


def old():
    torch.mm(p, W, out=gh)
    ops.batched_wgrad(p, h)
    ops.col_sum(p)


def t(fn, it=5):
    fn(); torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / it


def gh_blas():
    torch.mm(p, W, out=gh)


res = {"gh": t(gh_k), "gh_hipblaslt": t(gh_blas), "wgrad": t(wg_k), "old_total": t(old)}
ref = p @ W
gh_k()
torch.cuda.synchronize()
res_err = float((gh - ref).abs().max() / ref.abs().max())
print({k: f"{v:.2f}ms" for k, v in res.items()}, f"slab_rows={rows}", f"gh rel err {res_err:.2e}",
      flush=True)
