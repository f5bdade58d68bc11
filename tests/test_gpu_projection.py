"""regnn_type_project: the per-type input projection fused with the first aggregation's pre-scale
(model/REGCN.py:31-35 + layer/REGraphConv.py:56,73-76).

* h = x W^T + b against fp64 torch (ragged K, several node types at row offsets, fp32 and bf16);
* xs bit-identical to regnn_row_scale(h) with the same scale and dropout seed (the unfused path);
* REGCN with the fused projection equals the unfused composition (eval, and train with the same
  dropout seeds), values and every parameter gradient.
"""
import numpy as np
import pytest
import torch

from oracle import regnn_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("p", [0.0, 0.5, 0.3])
def test_type_project_kernel(dtype, p):
    from regnn_hip import _lib as L, ops
    g = torch.Generator(device=DEV)
    g.manual_seed(11)
    dims, rows = [128, 50, 20, 130], [3001, 517, 64, 1200]
    xs_in = [torch.randn(r, d, generator=g, device=DEV).to(dtype) for r, d in zip(rows, dims)]
    fcs = [torch.nn.Linear(d, 64).to(DEV) for d in dims]
    N = sum(rows)
    scale = torch.rand(N, generator=g, device=DEV) + 0.5
    drop = ops.drop_request(p, DEV) if p else None
    with torch.no_grad():
        h, xs = ops.type_project_prescale(fcs, xs_in, scale, drop)
    want = torch.cat([x.double() @ fc.weight.double().t() + fc.bias.double()
                      for x, fc in zip(xs_in, fcs)])
    tol = 1e-5 if dtype == torch.float32 else 1e-2          # bf16: one storage rounding of h
    err = float((h.double() - want).abs().max() / want.abs().max())
    assert err <= tol, f"projection rel err {err:.3e}"
    ref = torch.empty_like(h)
    seed, keep16, dscale = (None, 0, 1.0) if drop is None else (L.ptr(drop[0]), drop[1], drop[2])
    L.call("regnn_row_scale", L.ptr(h), L.ptr(scale), L.ptr(ref), N, 64, L.dtype_code(h), seed,
           keep16, dscale, None, None, L.stream())
    assert torch.equal(xs, ref), "xs differs from regnn_row_scale(h)"
    if drop is not None:
        mask = O.dropout_mask(int(drop[0].item()), N, 64, 16 // h.element_size(), keep16)
        kept = torch.from_numpy(mask).to(DEV).bool()
        assert torch.equal(xs == 0, ~kept | (h == 0))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("n,C,K", [(20000, 64, 128), (777, 33, 64), (5000, 64, 256), (31, 64, 128),
                                   (1000, 64, 192)])
def test_linear_wgrad(dtype, n, C, K):
    """regnn_linear_wgrad: (g^T x, colsum g) of a Linear's backward vs fp64, deterministic."""
    from regnn_hip import ops
    gen = torch.Generator(device=DEV)
    gen.manual_seed(n)
    g = torch.randn(n, C, generator=gen, device=DEV).to(dtype)
    x = torch.randn(n, K, generator=gen, device=DEV).to(dtype)
    gw, gb = ops.linear_wgrad(g, x)
    want_w = g.double().t() @ x.double()
    want_b = g.double().sum(0)
    rel = lambda a, b: float((a.double() - b).abs().max()) / max(1.0, float(b.abs().max()))
    assert gw.shape == (C, K) and gb.shape == (C,)
    assert rel(gw, want_w) <= 1e-5 and rel(gb, want_b) <= 1e-5
    gw2, gb2 = ops.linear_wgrad(g, x)
    assert torch.equal(gw, gw2) and torch.equal(gb, gb2)


@pytest.mark.parametrize("train", [False, True])
def test_regcn_fused_projection_matches_unfused(train):
    import torch.nn.functional as F
    from regnn_hip import nets, ops, synth
    import dgl
    gd = synth.mag_like(0.002, seed=3, device=DEV)
    g = dgl.DGLGraph((gd["src"], gd["dst"]), num_nodes=gd["N"])
    e_feat = gd["rel"].to(torch.int64)
    feats = synth.type_features(gd["counts"], {t: 128 for t in synth.NTYPES}, seed=1, device=DEV,
                                kind="mag")
    torch.manual_seed(0)
    net = nets.REGCN(g, gd["R"], 100.0, 64, 64, 349, 2, F.elu, 0.5,
                     [f.shape[1] for f in feats]).to(DEV)
    net.train(train)
    labels = torch.randint(0, 349, (gd["counts"]["paper"],), device=DEV)
    W, b = net.head()
    out = {}
    old = nets.FUSE_PROJECTION
    try:
        for fused in (False, True):
            nets.FUSE_PROJECTION = fused
            ops._DROP_CTR.clear()
            torch.manual_seed(5)                         # same dropout seeds in both runs
            net.zero_grad()
            h = net.embed(feats, e_feat)
            _, loss = ops.head_ce(h.float(), W, b, labels)
            loss.backward()
            out[fused] = (h.detach().clone(), float(loss),
                          {k: p.grad.clone() for k, p in net.named_parameters()
                           if p.grad is not None})
    finally:
        nets.FUSE_PROJECTION = old
    (h0, l0, g0), (h1, l1, g1) = out[False], out[True]
    rel = lambda a, b: float((a - b).abs().max()) / max(1.0, float(b.abs().max()))
    assert rel(h1, h0) <= 1e-5
    assert abs(l1 - l0) <= 1e-5 * max(1.0, abs(l0))
    assert g0.keys() == g1.keys()
    for k in g0:
        assert rel(g1[k], g0[k]) <= 1e-4, k


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("train", [False, True])
def test_regcn_projection_without_h_matches(dtype, train):
    """type_project_prescale(keep_h=False): the projection writes only the gathered rows xs and
    layer 0's backward reads xs for its node-norm and relation terms (REGNN_SELF_PRESCALED);
    loss and every gradient equal the run that stores h."""
    import torch.nn.functional as F
    from regnn_hip import nets, ops, synth
    import dgl
    gd = synth.mag_like(0.002, seed=4, device=DEV)
    g = dgl.DGLGraph((gd["src"], gd["dst"]), num_nodes=gd["N"])
    e_feat = gd["rel"].to(torch.int64)
    feats = [f.to(dtype) for f in synth.type_features(
        gd["counts"], {t: 128 for t in synth.NTYPES}, seed=1, device=DEV, kind="mag")]
    torch.manual_seed(0)
    net = nets.REGCN(g, gd["R"], 100.0, 64, 64, 349, 2, F.elu, 0.5,
                     [f.shape[1] for f in feats]).to(DEV)
    with torch.no_grad():                                # relation weights of both signs
        for layer in net.layers:
            layer.edge_weight.uniform_(-0.005, 0.015)
    net.train(train)
    labels = torch.randint(0, 349, (gd["counts"]["paper"],), device=DEV)
    W, b = net.head()
    out = {}
    old = dict(ops.PRESCALE)
    try:
        for mode in ("off", "auto"):
            ops.PRESCALE["self"] = mode
            ops._DROP_CTR.clear()
            torch.manual_seed(5)
            net.zero_grad()
            h = net.embed(feats, e_feat)
            _, loss = ops.head_ce(h, W, b, labels)
            loss.backward()
            out[mode] = (float(loss), {k: p.grad.clone() for k, p in net.named_parameters()
                                       if p.grad is not None})
    finally:
        ops.PRESCALE.update(old)
    (l0, g0), (l1, g1) = out["off"], out["auto"]
    assert l0 == l1
    rel = lambda a, b: float((a - b).abs().max()) / max(1e-3, float(b.abs().max()))
    assert g0.keys() == g1.keys()
    tol = 1e-5 if dtype == torch.float32 else 2e-2
    for k in g0:
        assert rel(g1[k], g0[k]) <= tol, k
