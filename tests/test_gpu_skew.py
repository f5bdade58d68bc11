"""GPU parity on power-law graphs whose hub rows take the long-segment path (chunk kernel + fixed-
order reduction tree), against the fp64 CPU oracle; several split/chunk settings force 1..4 tree
levels. Also: bitwise determinism and empty / isolated / self-loop-only rows."""
import numpy as np
import pytest
import torch

import _golden as G
from oracle import regnn_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL = 1e-5


def power_graph(N=4000, E=60000, R=7, seed=0, hub_edges=30000):
    rng = np.random.default_rng(seed)
    dst = np.minimum((rng.pareto(1.1, E) * 3).astype(np.int64), N - 1)
    src = rng.integers(0, N, E)
    # one explicit hub on both sides (in- and out-degree)
    src = np.concatenate([src, rng.integers(0, N, hub_edges), np.full(hub_edges // 2, 7)])
    dst = np.concatenate([dst, np.full(hub_edges, 3), rng.integers(0, N, hub_edges // 2)])
    # isolated destination rows 100..109 (no in-edges at all) -> deg 0 -> clamp
    keep = ~np.isin(dst, np.arange(100, 110))
    src, dst = src[keep], dst[keep]
    rel = rng.integers(1, R + 1, src.size)
    return src, dst, rel, N, R


def _oracle_layer(src, dst, rel, N, R, feat, ew, gout, norm=True):
    g = O.Graph(src, dst, N)
    o = O.REGraphConvOracle(100.0, feat.shape[1], feat.shape[1], norm=norm)
    out = o.forward(g, feat.astype(np.float64), rel, ew.astype(np.float64))
    gf, gr = o.backward(g, gout.astype(np.float64))
    return out, gf, gr["edge_weight"]


@pytest.mark.parametrize("split,chunk", [(256, 256), (32, 16), (8, 4), (64, 64)])
@pytest.mark.parametrize("F", [64, 32])
@pytest.mark.parametrize("order", ["edge", "source"])
def test_regraphconv_long_rows(split, chunk, F, order):
    """order="source": rows sorted by gathered id and chunks run in the scheduled order."""
    from layer import REGraphConv
    from regnn_hip.graph import RelGraph
    src, dst, rel, N, R = power_graph()
    rg = RelGraph(src, dst, N, DEV, split=split, chunk=chunk, order=order)
    assert rg.csr_plan.n_long > 0 and rg.csc_plan.n_long > 0
    assert (rg.csr_plan.chunk_sched is not None) == (order == "source")
    rng = np.random.default_rng(1)
    feat = rng.standard_normal((N, F)).astype(np.float32)
    ew = (rng.uniform(-0.5, 1.5, (R, 1)) / 100.0).astype(np.float32)
    gout = rng.standard_normal((N, F)).astype(np.float32)
    m = REGraphConv(R, 100.0, F, F, bias=False, weight=False).to(DEV)
    with torch.no_grad():
        m.edge_weight.copy_(torch.from_numpy(ew))
    x = torch.from_numpy(feat).to(DEV).requires_grad_(True)
    out = m(rg, x, torch.from_numpy(rel).to(DEV))
    out.backward(torch.from_numpy(gout).to(DEV))
    r_out, r_gf, r_gw = _oracle_layer(src, dst, rel, N, R, feat, ew, gout)
    for tag, got, want in (("out", out, r_out), ("grad_feat", x.grad, r_gf),
                           ("grad_edge_weight", m.edge_weight.grad, r_gw)):
        ok, err = G.close(got.detach().cpu().numpy(), want, TOL)
        assert ok, f"{tag} (split={split}, chunk={chunk}, levels={rg.csr_plan.n_levels}): {err:.3e}"


@pytest.mark.parametrize("order", ["edge", "source"])
def test_tree_levels_and_determinism(order):
    from layer import REGraphConv
    from regnn_hip.graph import RelGraph
    src, dst, rel, N, R = power_graph(hub_edges=70000)
    rg = RelGraph(src, dst, N, DEV, split=8, chunk=4, order=order)
    assert rg.csr_plan.n_levels >= 3, rg.csr_plan.n_levels
    rng = np.random.default_rng(2)
    x0 = torch.from_numpy(rng.standard_normal((N, 64)).astype(np.float32)).to(DEV)
    res = []
    for _ in range(2):
        m = REGraphConv(R, 100.0, 64, 64, bias=False, weight=False).to(DEV)
        x = x0.clone().requires_grad_(True)
        out = m(rg, x, torch.from_numpy(rel).to(DEV))
        out.square().sum().backward()
        res.append((out.detach(), x.grad, m.edge_weight.grad))
    for a, b in zip(*res):
        assert torch.equal(a, b)


def test_degenerate_rows():
    """empty graph rows, a node whose only edge is its self loop, relation id == R."""
    from layer import REGraphConv
    import dgl
    N, R = 6, 3
    src = np.array([0, 1, 2, 5, 5], dtype=np.int64)
    dst = np.array([1, 1, 2, 0, 4], dtype=np.int64)   # node 3 has no in-edges; 2 only a loop
    rel = np.array([1, 3, 2, 3, 1], dtype=np.int64)
    g = dgl.DGLGraph((src, dst), num_nodes=N).to(DEV)
    rng = np.random.default_rng(3)
    feat = rng.standard_normal((N, 64)).astype(np.float32)
    ew = np.array([[0.012], [-0.004], [0.009]], dtype=np.float32)
    gout = rng.standard_normal((N, 64)).astype(np.float32)
    m = REGraphConv(R, 100.0, 64, 64, bias=False, weight=False).to(DEV)
    with torch.no_grad():
        m.edge_weight.copy_(torch.from_numpy(ew))
    x = torch.from_numpy(feat).to(DEV).requires_grad_(True)
    out = m(g, x, torch.from_numpy(rel).to(DEV))
    out.backward(torch.from_numpy(gout).to(DEV))
    r_out, r_gf, r_gw = _oracle_layer(src, dst, rel, N, R, feat, ew, gout)
    assert G.close(out.detach().cpu().numpy(), r_out, TOL)[0]
    assert G.close(x.grad.cpu().numpy(), r_gf, TOL)[0]
    assert G.close(m.edge_weight.grad.cpu().numpy(), r_gw, TOL)[0]
    assert torch.all(out[3] == 0)


def test_relation_id_validation():
    from layer import REGraphConv
    import dgl
    g = dgl.DGLGraph((np.array([0, 1]), np.array([1, 0])), num_nodes=2).to(DEV)
    m = REGraphConv(2, 100.0, 8, 8, weight=False, bias=False).to(DEV)
    x = torch.zeros(2, 8, device=DEV)
    with pytest.raises(ValueError, match="relation ids"):
        m(g, x, torch.tensor([0, 1], device=DEV))      # id 0 would wrap to R-1 in the reference
    with pytest.raises(ValueError, match="relation ids"):
        m(g, x, torch.tensor([1, 3], device=DEV))      # id > R
