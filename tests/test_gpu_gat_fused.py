"""The fused GAT forward (regnn_gat_fused_fwd: scores + edge softmax + per-head SpMM in one
pass, layer/REGATConv.py:80-92) and its backward (attention re-formed from the log-sum-exp)
against the unfused HIP path (gat_attention + head_spmm, pinned on the golden REGATConv vectors)
on a power-law graph with hub rows, H=8 D=64 and H=4 D=16, with and without the relation bias.
fp32 at 1e-5 (relative to each tensor's max); the layer-level golden tests in test_gpu_layers.py
run REGATConv in eval mode, i.e. through the fused path."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _graph(N=3000, E=60000, R=7, seed=0):
    from regnn_hip.graph import RelGraph
    rng = np.random.default_rng(seed)
    dst = np.minimum((rng.pareto(1.1, E) * 3).astype(np.int64), N - 1)
    src = rng.integers(0, N, E)
    rel = rng.integers(1, R + 1, E)
    keep = np.arange(N)                               # every node has its self loop, as DGL graphs
    src = np.concatenate([src, keep]); dst = np.concatenate([dst, keep])
    rel = np.concatenate([rel, np.full(N, R)])
    rg = RelGraph(src, dst, N, DEV)
    return rg, torch.from_numpy(rel).to(DEV)


def _rel(x):
    return (x.abs().max().clamp(min=1.0)).item()


@pytest.mark.parametrize("H,D,use_ee", [(8, 64, True), (8, 64, False), (4, 16, True)])
def test_gat_fused_matches_unfused(H, D, use_ee):
    from regnn_hip import ops
    rg, e_feat = _graph()
    N = rg.n_dst
    g = torch.Generator(device=DEV).manual_seed(1)
    ft0 = torch.randn(N, H, D, generator=g, device=DEV)
    el0 = torch.randn(N, H, generator=g, device=DEV)
    er0 = torch.randn(N, H, generator=g, device=DEV)
    tab0 = torch.randn(7, H, generator=g, device=DEV) * 0.5 if use_ee else None
    pack = rg.rel_pack(e_feat, num_rel=7) if use_ee else None
    gy = torch.randn(N, H, D, generator=g, device=DEV)
    outs = []
    for fused in (False, True):
        ft, el, er = (t.clone().requires_grad_(True) for t in (ft0, el0, er0))
        tab = tab0.clone().requires_grad_(True) if use_ee else None
        if fused:
            y = ops.gat_fused(rg, el, er, ft, tab, pack, 0.2)
        else:
            y = ops.head_spmm(rg, ops.gat_attention(rg, el, er, tab, pack, 0.2), ft)
        y.backward(gy)
        outs.append([y.detach(), ft.grad, el.grad, er.grad] + ([tab.grad] if use_ee else []))
    for name, a, b in zip(["out", "g_ft", "g_el", "g_er", "g_tab"], outs[0], outs[1]):
        err = (a - b).abs().max().item() / _rel(a)
        assert err <= 1e-5, f"{name}: rel err {err:.3e}"
