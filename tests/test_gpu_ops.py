"""GPU checks of the operator layer: the generic DGL-front message passing (per-edge weights,
copy_u, mean), bf16 storage, the column-sum head kernel. References are plain fp64 torch
formulations of the same op on the host."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _graph(N=500, E=6000, seed=0):
    rng = np.random.default_rng(seed)
    src = rng.integers(0, N, E)
    dst = np.minimum((rng.pareto(1.0, E) * 4).astype(np.int64), N - 1)
    return src, dst, N


def _ref_spmm(src, dst, N, x, w):
    """fp64 y[v] = sum_e w[e] x[src[e]] with autograd."""
    s, d = torch.from_numpy(src), torch.from_numpy(dst)
    m = x[s] * w.view(-1, *([1] * (x.dim() - 1)))
    return torch.zeros((N,) + tuple(x.shape[1:]), dtype=x.dtype).index_add(0, d, m)


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / max(1.0, float(b.abs().max())))


@pytest.mark.parametrize("F", [1, 4, 64, 200])
def test_front_u_mul_e_sum(F):
    import dgl
    import dgl.function as fn
    src, dst, N = _graph()
    g = dgl.DGLGraph((src, dst), num_nodes=N).to(DEV)
    rng = np.random.default_rng(1)
    x0 = rng.standard_normal((N, F)).astype(np.float32)
    w0 = rng.standard_normal((src.size, 1)).astype(np.float32)
    gy = rng.standard_normal((N, F)).astype(np.float32)
    x = torch.from_numpy(x0).to(DEV).requires_grad_(True)
    w = torch.from_numpy(w0).to(DEV).requires_grad_(True)
    g.ndata["h"] = x
    g.edata["w"] = w
    g.update_all(fn.u_mul_e("h", "w", "m"), fn.sum("m", "y"))
    y = g.ndata["y"]
    y.backward(torch.from_numpy(gy).to(DEV))
    xr = torch.from_numpy(x0).double().requires_grad_(True)
    wr = torch.from_numpy(w0).double().requires_grad_(True)
    yr = _ref_spmm(src, dst, N, xr, wr.view(-1))
    yr.backward(torch.from_numpy(gy).double())
    assert _rel(y, yr) < 1e-5
    assert _rel(x.grad, xr.grad) < 1e-5
    assert _rel(w.grad, wr.grad) < 1e-5


def test_front_copy_u_mean_and_heads():
    import dgl
    import dgl.function as fn
    src, dst, N = _graph(seed=2)
    g = dgl.DGLGraph((src, dst), num_nodes=N).to(DEV)
    rng = np.random.default_rng(3)
    x0 = rng.standard_normal((N, 4, 32)).astype(np.float32)
    a0 = rng.random((src.size, 4, 1)).astype(np.float32)
    x = torch.from_numpy(x0).to(DEV)
    g.ndata["h"] = x
    g.update_all(fn.copy_u("h", "m"), fn.mean("m", "y"))
    yr = _ref_spmm(src, dst, N, torch.from_numpy(x0).double(), torch.ones(src.size, dtype=torch.float64))
    cnt = torch.bincount(torch.from_numpy(dst), minlength=N).clamp(min=1).double()
    assert _rel(g.ndata["y"], yr / cnt.view(-1, 1, 1)) < 1e-5
    g.edata["a"] = torch.from_numpy(a0).to(DEV)
    g.update_all(fn.u_mul_e("h", "a", "m"), fn.sum("m", "z"))
    zr = torch.stack([_ref_spmm(src, dst, N, torch.from_numpy(x0[:, h]).double(),
                                torch.from_numpy(a0[:, h, 0]).double()) for h in range(4)], 1)
    assert _rel(g.ndata["z"], zr) < 1e-5


def test_bf16_storage_close_to_fp32():
    from regnn_hip import ops
    from regnn_hip.graph import RelGraph
    src, dst, N = _graph(2000, 30000, seed=4)
    rg = RelGraph(src, dst, N, DEV, split=32, chunk=32)
    rng = np.random.default_rng(5)
    R = 5
    rel = torch.from_numpy(rng.integers(1, R + 1, src.size)).to(DEV)
    pack = rg.rel_pack(rel, R)
    tab = torch.rand(R, 1, device=DEV) + 0.5
    norm = ops.degree_norm(rg, pack, tab)
    x = torch.randn(N, 64, device=DEV)
    y32 = ops.re_spmm(rg, x, tab, pack, pre=norm, post=norm)
    y16 = ops.re_spmm(rg, x.bfloat16(), tab, pack, pre=norm, post=norm)
    assert y16.dtype == torch.bfloat16
    assert _rel(y16.float(), y32) < 2e-2
    # backward in bf16 storage
    xb = x.bfloat16().requires_grad_(True)
    ops.re_spmm(rg, xb, tab, pack, pre=norm.detach(), post=norm.detach()).float().sum().backward()
    xf = x.clone().requires_grad_(True)
    ops.re_spmm(rg, xf, tab, pack, pre=norm.detach(), post=norm.detach()).sum().backward()
    assert _rel(xb.grad.float(), xf.grad) < 2e-2


@pytest.mark.parametrize("rows,cols", [(1, 3), (1000, 349), (3_000_001, 64)])
def test_col_sum(rows, cols):
    from regnn_hip import ops
    x = torch.randn(rows, cols, device=DEV)
    got = ops.col_sum(x)
    want = x.double().sum(0)
    assert _rel(got, want) < 1e-5
    assert torch.equal(got, ops.col_sum(x))      # deterministic


@pytest.mark.parametrize("rows,width", [(2048, 22880), (300, 8256), (255, 5000), (2048, 4096),
                                        (1000, 4095), (33, 9000),
                                        # narrow: relation tables over 4096 rows
                                        (4096, 11), (4096, 16), (4096, 17), (4096, 32), (5000, 1),
                                        (3, 14), (4096, 33)])
@pytest.mark.parametrize("accumulate", [False, True])
def test_rel_reduce_wide(rows, width, accumulate):
    """regnn_rel_reduce on wide slabs (the in-place two-stage split for tall ones) and narrow ones
    (relation tables): fixed-order column sums, deterministic."""
    from regnn_hip import _lib as L
    g = torch.Generator(device=DEV).manual_seed(rows + width)
    slab = torch.randn(rows, width, device=DEV, generator=g)
    base = torch.randn(width, device=DEV, generator=g)
    want = slab.double().sum(0) + (base.double() if accumulate else 0)
    outs = []
    for _ in range(2):
        s = slab.clone()
        out = base.clone()
        L.call("regnn_rel_reduce", L.ptr(s), rows, width, L.ptr(out), int(accumulate), L.stream())
        outs.append(out)
    assert _rel(outs[0], want) < 1e-5
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("bias", [True, False])
@pytest.mark.parametrize("N,D,C,n", [(5000, 64, 349, 1800),     # fused MFMA head, 11 col tiles
                                     (1001, 64, 3, 1001),       # 1 col tile, every row a loss row
                                     (77, 64, 384, 5),          # 12 col tiles, ragged tile tails
                                     (300, 64, 33, 31),     # C just past one tile
                                     (640, 32, 349, 100),       # K != 64: GEMM + softmax_xent
                                     (200_000, 64, 349, 150_000)])  # many rows per wgrad block
@pytest.mark.parametrize("mode", ["z", "p"])
def test_head_ce_matches_autograd(bias, N, D, C, n, mode, monkeypatch):
    """ops.head_ce == out_lin over all rows + cross_entropy(logits[:n], y) (run_regnn.py:146-148),
    with p re-formed from the logits rows in the backward (z, the default) or stored (p)."""
    from regnn_hip import ops
    monkeypatch.setitem(ops.HEAD, "p", mode)
    torch.manual_seed(0)
    h0 = torch.randn(N, D, device=DEV)
    W0 = torch.randn(C, D, device=DEV) * 0.1
    b0 = torch.randn(C, device=DEV) * 0.1 if bias else None
    y = torch.randint(0, C, (n,), device=DEV)
    h, W = h0.clone().requires_grad_(True), W0.clone().requires_grad_(True)
    b = b0.clone().requires_grad_(True) if bias else None
    logits, loss = ops.head_ce(h, W, b, y)
    (loss * 0.75).backward()
    hr, Wr = h0.double().requires_grad_(True), W0.double().requires_grad_(True)
    br = b0.double().requires_grad_(True) if bias else None
    lr = hr @ Wr.t() + (br if bias else 0)
    lossr = torch.nn.functional.cross_entropy(lr[:n], y)
    (lossr * 0.75).backward()
    assert _rel(logits, lr) < 1e-5 and abs(loss.item() - lossr.item()) < 1e-5
    assert _rel(h.grad, hr.grad) < 1e-5 and _rel(W.grad, Wr.grad) < 1e-5
    if bias:
        assert _rel(b.grad, br.grad) < 1e-5


@pytest.mark.parametrize("C,n", [(349, 1500), (40, 7)])
def test_head_ce_logits_modified_in_place(C, n):
    """z mode re-forms p from the logits rows it returned: a caller that overwrites them before
    backward must still get the gradients of the loss it was given (the op recomputes p from h)."""
    from regnn_hip import ops
    assert ops.HEAD["p"] == "z"
    torch.manual_seed(3)
    N = 3000
    h0, W0, b0 = torch.randn(N, 64, device=DEV), torch.randn(C, 64, device=DEV) * 0.1, \
        torch.randn(C, device=DEV) * 0.1
    y = torch.randint(0, C, (n,), device=DEV)
    grads = []
    for clobber in (False, True):
        h, W, b = (t.clone().requires_grad_(True) for t in (h0, W0, b0))
        logits, loss = ops.head_ce(h, W, b, y)
        if clobber:
            logits.mul_(0.0).add_(7.0)
        loss.backward()
        grads.append((h.grad, W.grad, b.grad))
    hr, Wr, br = (t.double().requires_grad_(True) for t in (h0, W0, b0))
    torch.nn.functional.cross_entropy((hr @ Wr.t() + br)[:n], y).backward()
    for got in grads:
        assert _rel(got[0], hr.grad) < 1e-5 and _rel(got[1], Wr.grad) < 1e-5
        assert _rel(got[2], br.grad) < 1e-5


@pytest.mark.parametrize("N,H,D", [(1000, 8, 64), (77, 1, 3), (300, 4, 20)])
def test_attn_dots_matches_autograd(N, H, D):
    """ops.attn_dots == ((ft * attn_l).sum(-1), (ft * attn_r).sum(-1)) (layer/REGATConv.py:68-69),
    values and gradients of ft / attn_l / attn_r."""
    from regnn_hip import ops
    torch.manual_seed(1)
    ft0 = torch.randn(N, H, D, device=DEV)
    al0, ar0 = torch.randn(1, H, D, device=DEV), torch.randn(1, H, D, device=DEV)
    ft, al, ar = (t.clone().requires_grad_(True) for t in (ft0, al0, ar0))
    el, er = ops.attn_dots(ft, al, ar)
    gl, gr = torch.randn(N, H, device=DEV), torch.randn(N, H, device=DEV)
    (el * gl + er * gr).sum().backward()
    ftr, alr, arr = (t.double().requires_grad_(True) for t in (ft0, al0, ar0))
    elr, err = (ftr * alr).sum(-1), (ftr * arr).sum(-1)
    (elr * gl.double() + err * gr.double()).sum().backward()
    assert _rel(el, elr) < 1e-5 and _rel(er, err) < 1e-5
    assert _rel(ft.grad, ftr.grad) < 1e-5
    assert _rel(al.grad, alr.grad) < 1e-5 and _rel(ar.grad, arr.grad) < 1e-5


@pytest.mark.parametrize("clobber", [False, True])
def test_head_ce_bf16_rows_match_widened(clobber):
    """head_ce on bf16 rows (read as they are, regnn_head_fwd_lse / _bwd_z dtype 1) equals head_ce
    on their fp32 widening: logits and loss bit-identical (bf16 values are exact in the first
    bf16x6 split), gradients equal up to the final bf16 rounding of d h; also when the logits
    are overwritten before backward (p recomputed from the rows)."""
    from regnn_hip import ops
    torch.manual_seed(4)
    N, n, C = 5000, 1800, 349
    hb = torch.randn(N, 64, device=DEV).bfloat16()
    W0, b0 = torch.randn(C, 64, device=DEV) * 0.1, torch.randn(C, device=DEV) * 0.1
    y = torch.randint(0, C, (n,), device=DEV)
    out = {}
    for dt in (torch.bfloat16, torch.float32):
        h = hb.to(dt).clone().requires_grad_(True)
        W, b = W0.clone().requires_grad_(True), b0.clone().requires_grad_(True)
        logits, loss = ops.head_ce(h, W, b, y)
        lg = logits.clone()
        if clobber:
            logits.fill_(3.0)
        loss.backward()
        assert h.grad.dtype == dt
        out[dt] = (lg, loss.detach(), h.grad.float(), W.grad, b.grad)
    a, r = out[torch.bfloat16], out[torch.float32]
    assert torch.equal(a[0], r[0]) and torch.equal(a[1], r[1])
    assert torch.equal(a[2], r[2].bfloat16().float())
    assert _rel(a[3], r[3]) < 1e-6 and _rel(a[4], r[4]) < 1e-6


@pytest.mark.parametrize("seed", [0, 1])
def test_degree_histogram_matches_walk(seed):
    """regnn_degree_cnt / _bwd (per-row relation histogram) == regnn_degree / _bwd (relation-id
    walk): weighted degrees, norms and the relation-table gradient, on a graph with long rows."""
    import numpy as np
    from regnn_hip import ops
    from regnn_hip.graph import RelGraph
    rng = np.random.default_rng(seed)
    N, E, R = 3000, 60000, 11
    src = rng.integers(0, N, E)
    dst = np.where(rng.random(E) < 0.2, rng.integers(0, 3, E), rng.integers(0, N, E))
    rel = rng.integers(1, R + 1, E)
    rg = RelGraph(src, dst, N, DEV)
    pack = rg.rel_pack(torch.from_numpy(rel).to(DEV), num_rel=R)
    assert rg.csr_plan.n_long > 0
    tab0 = torch.rand(R, 1, device=DEV) * 2 - 0.5
    gn = torch.randn(N, device=DEV)
    out = {}
    old = ops.DEGREE["mode"]
    try:
        for mode in ("hist", "off"):
            ops.DEGREE["mode"] = mode
            tab = tab0.clone().requires_grad_(True)
            norm = ops.degree_norm(rg, pack, tab)
            (norm * gn).sum().backward()
            out[mode] = (norm.detach(), tab.grad)
    finally:
        ops.DEGREE["mode"] = old
    assert _rel(out["hist"][0], out["off"][0]) < 1e-6
    assert _rel(out["hist"][1], out["off"][1]) < 1e-5
