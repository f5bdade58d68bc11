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


def _hub_graph(N=4000, E=120000, R=7, seed=3):
    """hubs on both sides: destinations Pareto(1.1) (rows of ~10^4 in-edges, the CSR chunk path)
    and half the sources Pareto too (the CSC chunk path of the transposed kernels)."""
    from regnn_hip.graph import RelGraph
    rng = np.random.default_rng(seed)
    dst = np.minimum((rng.pareto(1.1, E) * 3).astype(np.int64), N - 1)
    src = rng.integers(0, N, E)
    half = rng.random(E) < 0.5
    src[half] = np.minimum((rng.pareto(1.1, int(half.sum())) * 5).astype(np.int64), N - 1)
    rel = rng.integers(1, R + 1, E)
    keep = np.arange(N)
    src = np.concatenate([src, keep]); dst = np.concatenate([dst, keep])
    rel = np.concatenate([rel, np.full(N, R)])
    rg = RelGraph(src, dst, N, DEV)
    return rg, torch.from_numpy(rel).to(DEV)


def _gat_reference(rg, rel_csr, el, er, tab, ft, slope):
    """fp64 torch restatement of layer/REGATConv.py:80-92 over the CSR edge list."""
    ptr = rg.csr_ptr.long()
    src = rg.csr_idx.long()
    dst = torch.repeat_interleave(torch.arange(rg.n_dst, device=DEV), ptr[1:] - ptr[:-1])
    s = el[src] + er[dst] + (tab[rel_csr.long()] if tab is not None else 0.0)
    s = torch.nn.functional.leaky_relu(s, slope)
    H = s.shape[1]
    m = torch.full((rg.n_dst, H), -torch.inf, dtype=s.dtype, device=DEV)
    m = m.scatter_reduce(0, dst[:, None].expand(-1, H), s, reduce="amax", include_self=True)
    ex = torch.exp(s - m[dst])
    den = torch.zeros(rg.n_dst, H, dtype=s.dtype, device=DEV).index_add(0, dst, ex)
    a = ex / den[dst]
    out = torch.zeros(rg.n_dst, H, ft.shape[2], dtype=s.dtype, device=DEV)
    return out.index_add(0, dst, a[:, :, None] * ft[src])


@pytest.mark.parametrize("fused", [True, False])
def test_gat_long_rows_vs_fp64(fused):
    """rows far past the chunk split on both sides (regnn_seg_plan: chunk partials + fixed-order
    tree for the online softmax, the per-head sums, the softmax backward's dots and sums and the
    segment sums): forward and every gradient against an fp64 restatement at 1e-5."""
    from regnn_hip import ops
    rg, e_feat = _hub_graph()
    assert rg.csr_plan.n_long > 0 and rg.csc_plan.n_long > 0
    deg = (rg.csr_ptr[1:] - rg.csr_ptr[:-1]).max().item()
    assert deg > 20 * rg.csr_plan.chunk                 # a segment of many chunks (tree levels)
    N, H, D = rg.n_dst, 8, 32
    g = torch.Generator(device=DEV).manual_seed(2)
    ft0 = torch.randn(N, H, D, generator=g, device=DEV)
    el0 = torch.randn(N, H, generator=g, device=DEV)
    er0 = torch.randn(N, H, generator=g, device=DEV)
    tab0 = torch.randn(7, H, generator=g, device=DEV) * 0.5
    pack = rg.rel_pack(e_feat, num_rel=7)
    gy = torch.randn(N, H, D, generator=g, device=DEV)
    ft, el, er, tab = (t.clone().requires_grad_(True) for t in (ft0, el0, er0, tab0))
    if fused:
        y = ops.gat_fused(rg, el, er, ft, tab, pack, 0.2)
    else:
        y = ops.head_spmm(rg, ops.gat_attention(rg, el, er, tab, pack, 0.2), ft)
    y.backward(gy)
    got = [y.detach(), ft.grad, el.grad, er.grad, tab.grad]
    ref_in = [t.double().clone().requires_grad_(True) for t in (el0, er0, tab0, ft0)]
    yr = _gat_reference(rg, pack.rel_csr, *ref_in, 0.2)
    yr.backward(gy.double())
    want = [yr.detach(), ref_in[3].grad, ref_in[0].grad, ref_in[1].grad, ref_in[2].grad]
    for name, a, b in zip(["out", "g_ft", "g_el", "g_er", "g_tab"], got, want):
        err = (a.double() - b).abs().max().item() / _rel(b)
        assert err <= 1e-5, f"{name}: rel err {err:.3e}"


@pytest.mark.parametrize("H,D,hub", [(8, 64, False), (8, 64, True), (4, 16, False), (2, 8, True),
                                     (8, 32, False), (4, 4, False), (2, 128, False),
                                     (2, 256, False)])
def test_gat_fused_el_reformed_bitwise(H, D, hub):
    """attn_l passed: the forward re-forms el from the gathered rows (regnn_attn_dots_fwd's
    summation order) instead of reading it; outputs and gradients bitwise those of the el-reading
    kernel (D = 128 on 16-lane rows: the el-reading kernel runs either way)."""
    from regnn_hip import ops
    rg, e_feat = (_hub_graph() if hub else _graph())
    N = rg.n_dst
    g = torch.Generator(device=DEV).manual_seed(5)
    ft0 = torch.randn(N, H, D, generator=g, device=DEV)
    al0 = torch.randn(1, H, D, generator=g, device=DEV) * 0.3
    ar0 = torch.randn(1, H, D, generator=g, device=DEV) * 0.3
    tab0 = torch.randn(7, H, generator=g, device=DEV) * 0.5
    pack = rg.rel_pack(e_feat, num_rel=7)
    gy = torch.randn(N, H, D, generator=g, device=DEV)
    outs = []
    for pass_al in (False, True):
        ft, al, ar, tab = (t.clone().requires_grad_(True) for t in (ft0, al0, ar0, tab0))
        el, er = ops.attn_dots(ft, al, ar)
        y = ops.gat_fused(rg, el, er, ft, tab, pack, 0.2, attn_l=al if pass_al else None)
        y.backward(gy)
        outs.append([y.detach(), ft.grad, al.grad, ar.grad, tab.grad])
    for name, a, b in zip(["out", "g_ft", "g_al", "g_ar", "g_tab"], outs[0], outs[1]):
        assert torch.equal(a, b), f"{name}: max diff {(a - b).abs().max().item():.3e}"


def test_attn_dots_vec_order_matches_fp64():
    """regnn_attn_dots_fwd in the lane order the fused forward re-forms el in, against fp64."""
    from regnn_hip import ops
    g = torch.Generator(device=DEV).manual_seed(6)
    for H, D in [(8, 64), (4, 16), (3, 4), (2, 12)]:
        ft = torch.randn(5000, H, D, generator=g, device=DEV)
        al = torch.randn(1, H, D, generator=g, device=DEV)
        ar = torch.randn(1, H, D, generator=g, device=DEV)
        el, er = ops.attn_dots(ft, al, ar)
        rl = (ft.double() * al.double()).sum(-1)
        rr = (ft.double() * ar.double()).sum(-1)
        assert (el.double() - rl).abs().max().item() <= 1e-5 * max(1.0, rl.abs().max().item())
        assert (er.double() - rr).abs().max().item() <= 1e-5 * max(1.0, rr.abs().max().item())


def _gatv2_reference(rg, rel_csr, fs, fd, att, tab, ft, slope, global_max=False):
    """fp64 torch restatement of layer/REGATv2Conv.py:139-163 (GATv2 score, relation bias,
    per-destination softmax; global_max: mag/utils.py:45-57) and the per-head aggregation."""
    ptr = rg.csr_ptr.long()
    src = rg.csr_idx.long()
    dst = torch.repeat_interleave(torch.arange(rg.n_dst, device=DEV), ptr[1:] - ptr[:-1])
    e = torch.nn.functional.leaky_relu(fs[src] + fd[dst], slope)             # [E, H, D]
    s = (e * att).sum(-1)
    if tab is not None:
        s = s + tab[rel_csr.long()]
    H = s.shape[1]
    if global_max:
        ex = torch.exp(s - s.max())
        den = torch.zeros(rg.n_dst, H, dtype=s.dtype, device=DEV).index_add(0, dst, ex)
        a = ex / (den[dst] + 1e-16)
    else:
        m = torch.full((rg.n_dst, H), -torch.inf, dtype=s.dtype, device=DEV)
        m = m.scatter_reduce(0, dst[:, None].expand(-1, H), s, reduce="amax", include_self=True)
        ex = torch.exp(s - m[dst])
        den = torch.zeros(rg.n_dst, H, dtype=s.dtype, device=DEV).index_add(0, dst, ex)
        a = ex / den[dst]
    out = torch.zeros(rg.n_dst, H, ft.shape[2], dtype=s.dtype, device=DEV)
    return out.index_add(0, dst, a[:, :, None] * ft[src])


@pytest.mark.parametrize("global_max", [False, True])
def test_gatv2_long_rows_vs_fp64(global_max):
    """GATv2's score SDDMM, its two backward passes and the edge softmax on
    rows far past the chunk split on both sides (regnn_seg_plan chunks + fixed-order tree):
    forward and every gradient against an fp64 restatement at 1e-5."""
    from regnn_hip import ops
    rg, e_feat = _hub_graph()
    assert rg.csr_plan.n_long > 0 and rg.csc_plan.n_long > 0
    N, H, D = rg.n_dst, 4, 16
    g = torch.Generator(device=DEV).manual_seed(7)
    fs0 = torch.randn(N, H, D, generator=g, device=DEV) * 0.5
    fd0 = torch.randn(N, H, D, generator=g, device=DEV) * 0.5
    att0 = torch.randn(1, H, D, generator=g, device=DEV) * 0.3
    tab0 = torch.randn(7, H, generator=g, device=DEV) * 0.5
    ft0 = torch.randn(N, H, D, generator=g, device=DEV)
    pack = rg.rel_pack(e_feat, num_rel=7)
    gy = torch.randn(N, H, D, generator=g, device=DEV)
    fs, fd, att, tab, ft = (t.clone().requires_grad_(True) for t in (fs0, fd0, att0, tab0, ft0))
    s = ops.gatv2_scores(rg, fs, fd, att, 0.2)
    a = ops.edge_softmax_logits(rg, s, tab, pack, global_max)
    y = ops.head_spmm(rg, a, ft)
    y.backward(gy)
    got = [y.detach(), fs.grad, fd.grad, att.grad, tab.grad, ft.grad]
    ref_in = [t.double().clone().requires_grad_(True) for t in (fs0, fd0, att0, tab0, ft0)]
    yr = _gatv2_reference(rg, pack.rel_csr, *ref_in, 0.2, global_max)
    yr.backward(gy.double())
    want = [yr.detach()] + [t.grad for t in ref_in]
    for name, x, w in zip(["out", "g_fs", "g_fd", "g_att", "g_tab", "g_ft"], got, want):
        err = (x.double() - w).abs().max().item() / _rel(w)
        assert err <= 1e-5, f"{name}: rel err {err:.3e}"


def _single_chunk_graph(N=3000, E=30000, R=7, seed=4):
    """long rows that are each ONE chunk on both sides (split 32 < degree <= chunk 256): the plan
    has chunks but no tree levels (n_levels == 0), its final rows the chunk rows themselves."""
    from regnn_hip.graph import RelGraph
    rng = np.random.default_rng(seed)
    dst = rng.integers(0, N, E)
    src = rng.integers(0, N, E)
    hubs = rng.choice(N, 40, replace=False)
    hd = np.repeat(hubs[:20], 150)                      # 20 destinations with 150+ in-edges
    hs = np.repeat(hubs[20:], 170)                      # 20 sources with 170+ out-edges
    src = np.concatenate([src, rng.integers(0, N, hd.size), hs])
    dst = np.concatenate([dst, hd, rng.integers(0, N, hs.size)])
    rel = rng.integers(1, R + 1, src.size)
    keep = np.arange(N)
    src = np.concatenate([src, keep]); dst = np.concatenate([dst, keep])
    rel = np.concatenate([rel, np.full(N, R)])
    rg = RelGraph(src, dst, N, DEV, split=32, chunk=256)
    return rg, torch.from_numpy(rel).to(DEV)


@pytest.mark.parametrize("kind", ["gat_fused", "gat", "gatv2"])
def test_attention_single_chunk_long_rows_vs_fp64(kind):
    """a plan whose long segments are one chunk each (n_levels == 0) runs -- the GAT /
    GATv2 score, softmax and aggregation kernels read the chunk rows as the final rows -- and
    matches the fp64 restatement at 1e-5, forward and every gradient."""
    from regnn_hip import ops
    rg, e_feat = _single_chunk_graph()
    for plan in (rg.csr_plan, rg.csc_plan):
        assert plan.n_long > 0 and plan.n_chunk == plan.n_long and plan.n_levels == 0
    N = rg.n_dst
    g = torch.Generator(device=DEV).manual_seed(9)
    pack = rg.rel_pack(e_feat, num_rel=7)
    if kind.startswith("gat") and kind != "gatv2":
        H, D = 4, 16
        ft0 = torch.randn(N, H, D, generator=g, device=DEV)
        el0 = torch.randn(N, H, generator=g, device=DEV)
        er0 = torch.randn(N, H, generator=g, device=DEV)
        tab0 = torch.randn(7, H, generator=g, device=DEV) * 0.5
        gy = torch.randn(N, H, D, generator=g, device=DEV)
        ft, el, er, tab = (t.clone().requires_grad_(True) for t in (ft0, el0, er0, tab0))
        if kind == "gat_fused":
            y = ops.gat_fused(rg, el, er, ft, tab, pack, 0.2)
        else:
            y = ops.head_spmm(rg, ops.gat_attention(rg, el, er, tab, pack, 0.2), ft)
        y.backward(gy)
        got = [y.detach(), ft.grad, el.grad, er.grad, tab.grad]
        ref_in = [t.double().clone().requires_grad_(True) for t in (el0, er0, tab0, ft0)]
        yr = _gat_reference(rg, pack.rel_csr, *ref_in, 0.2)
        yr.backward(gy.double())
        want = [yr.detach(), ref_in[3].grad, ref_in[0].grad, ref_in[1].grad, ref_in[2].grad]
    else:
        H, D = 4, 16
        fs0 = torch.randn(N, H, D, generator=g, device=DEV) * 0.5
        fd0 = torch.randn(N, H, D, generator=g, device=DEV) * 0.5
        att0 = torch.randn(1, H, D, generator=g, device=DEV) * 0.3
        tab0 = torch.randn(7, H, generator=g, device=DEV) * 0.5
        ft0 = torch.randn(N, H, D, generator=g, device=DEV)
        gy = torch.randn(N, H, D, generator=g, device=DEV)
        fs, fd, att, tab, ft = (t.clone().requires_grad_(True)
                                for t in (fs0, fd0, att0, tab0, ft0))
        s = ops.gatv2_scores(rg, fs, fd, att, 0.2)
        y = ops.head_spmm(rg, ops.edge_softmax_logits(rg, s, tab, pack, False), ft)
        y.backward(gy)
        got = [y.detach(), fs.grad, fd.grad, att.grad, tab.grad, ft.grad]
        ref_in = [t.double().clone().requires_grad_(True) for t in (fs0, fd0, att0, tab0, ft0)]
        yr = _gatv2_reference(rg, pack.rel_csr, *ref_in, 0.2, False)
        yr.backward(gy.double())
        want = [yr.detach()] + [t.grad for t in ref_in]
    for i, (x, w) in enumerate(zip(got, want)):
        err = (x.double() - w).abs().max().item() / _rel(w)
        assert err <= 1e-5, f"{kind} output {i}: rel err {err:.3e}"
