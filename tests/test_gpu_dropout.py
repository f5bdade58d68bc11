"""Fused dropout of the SpMM gather (regnn_spmm_fwd_dropout / regnn_spmm_bwd_dropout): outputs
and every gradient equal the unfused composition dropout -> pre-scale -> SpMM -> post-scale
(+bias) with the mask restated in oracle.regnn_oracle.dropout_mask, computed by torch autograd in
fp64 on the CPU; plus the keep rate and the layer / model wiring."""
import numpy as np
import pytest
import torch

from oracle import regnn_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _graph(n=700, m=9000, R=6, hub=600, seed=0):
    rng = np.random.default_rng(seed)
    src = rng.integers(0, n, m)
    dst = rng.integers(0, n, m)
    dst[:hub] = 3                                     # one row through the chunked path
    rel = rng.integers(1, R + 1, m)
    return src, dst, rel, n, R


@pytest.mark.parametrize("dtype,F", [(torch.float32, 64), (torch.bfloat16, 128),
                                     (torch.bfloat16, 64), (torch.float32, 32)])
@pytest.mark.parametrize("p", [0.5, 0.3, 0.75, 0.0])
@pytest.mark.parametrize("prescale", ["on", "off"])
def test_fused_dropout_matches_masked_composition(dtype, F, p, prescale):
    """prescale "on": regnn_row_scale forms norm * drop(x) per row and the gather reads it;
    "off": the gather masks and scales every edge's row (regnn_spmm_fwd_dropout)."""
    from regnn_hip import ops
    old = dict(ops.PRESCALE)
    ops.PRESCALE.update(mode=prescale, bwd=prescale)
    try:
        _check_dropout_composition(dtype, F, p)
    finally:
        ops.PRESCALE.update(old)


def _check_dropout_composition(dtype, F, p):
    from regnn_hip import ops
    from regnn_hip.graph import RelGraph
    src, dst, rel, n, R = _graph()
    rg = RelGraph(src, dst, n, DEV)
    pack = rg.rel_pack(torch.from_numpy(rel).to(DEV), num_rel=R)
    g = torch.Generator().manual_seed(1)
    x = torch.randn(n, F, generator=g).to(dtype)
    tab = (torch.rand(R, 1, generator=g) + 0.2)
    norm = torch.rand(n, generator=g) + 0.5
    bias = torch.randn(F, generator=g)
    gy = torch.randn(n, F, generator=g).to(dtype)
    seed = torch.tensor([0x1234_5678_9ABC_DEF1], dtype=torch.int64, device=DEV)

    xd = x.to(DEV).requires_grad_(True)
    td = tab.to(DEV).requires_grad_(True)
    nd = norm.to(DEV).requires_grad_(True)
    bd = bias.to(DEV).requires_grad_(True)
    y = ops.re_spmm(rg, xd, td, pack, pre=nd, post=nd, bias=bd, dropout=p, drop_seed=seed)
    y.backward(gy.to(DEV))

    keep16 = int(round((1 - p) * 65536))
    mask = torch.from_numpy(O.dropout_mask(int(seed.item()), n, F, 16 // x.element_size(), keep16))
    X = x.double().requires_grad_(True)
    T = tab.double().requires_grad_(True)
    Nn = norm.double().requires_grad_(True)
    B = bias.double().requires_grad_(True)
    w = T[torch.from_numpy(rel - 1), 0]                          # the table as given
    A = torch.sparse_coo_tensor(torch.from_numpy(np.stack([dst, src])), w, (n, n))
    xin = X * mask / (1 - p) * Nn[:, None]
    Y = Nn[:, None] * torch.sparse.mm(A, xin) + B
    Y.backward(gy.double())
    tol = 1e-5 if dtype == torch.float32 else 2e-2
    scale = lambda t: max(1.0, float(t.abs().max()))
    for tag, a, b in (("y", y, Y), ("gx", xd.grad, X.grad), ("gtab", td.grad, T.grad),
                      ("gnorm", nd.grad, Nn.grad), ("gbias", bd.grad, B.grad)):
        err = float((a.detach().double().cpu() - b.detach()).abs().max()) / scale(b)
        assert err <= tol, f"{tag}: rel err {err:.3e}"
    kept = float(mask.mean())
    assert abs(kept - (1 - p)) < 0.01


def test_regcn_training_uses_fused_dropout():
    """REGCN in train mode: layer 0's feat_dropout and the model dropout + layer 1's feat_dropout
    run inside the SpMM gathers (no torch dropout kernels); eval mode is deterministic."""
    import torch.nn.functional as F
    import dgl
    from regnn_hip import nets, ops
    src, dst, rel, n, R = _graph(seed=3)
    loops = np.arange(n)
    g = dgl.DGLGraph((np.concatenate([src, loops]), np.concatenate([dst, loops])), num_nodes=n)
    g = g.to(DEV)
    e_feat = torch.from_numpy(np.concatenate([rel, np.full(n, R)])).to(DEV)
    torch.manual_seed(0)
    net = nets.REGCN(g, R, 100.0, 64, 64, 3, 2, F.elu, 0.5, [16]).to(DEV)
    feats = [torch.randn(n, 16, device=DEV)]
    calls = []
    orig = torch.nn.functional.dropout
    torch.nn.functional.dropout = lambda *a, **k: calls.append(1) or orig(*a, **k)
    try:
        net.train()
        h1 = net.embed(feats, e_feat)
        h2 = net.embed(feats, e_feat)
        h1.sum().backward()
    finally:
        torch.nn.functional.dropout = orig
    assert not calls, "torch dropout ran: the dropout was not fused"
    assert not torch.equal(h1, h2)                     # a fresh mask per call
    assert all(torch.isfinite(p.grad).all() for p in net.parameters() if p.grad is not None)
    net.eval()
    e1, e2 = net.embed(feats, e_feat), net.embed(feats, e_feat)
    assert torch.equal(e1, e2)


def test_regcn_bf16_storage_matches_fp32():
    """bench --dtype bf16 (BASELINE configs[1]): bf16 feature storage, fp32 master weights and
    accumulation; logits and weight gradients within bf16 tolerance of the fp32 model."""
    import torch.nn.functional as F
    import dgl
    from regnn_hip import nets, ops
    src, dst, rel, n, R = _graph(seed=5)
    loops = np.arange(n)
    g = dgl.DGLGraph((np.concatenate([src, loops]), np.concatenate([dst, loops])),
                     num_nodes=n).to(DEV)
    e_feat = torch.from_numpy(np.concatenate([rel, np.full(n, R)])).to(DEV)
    torch.manual_seed(0)
    net = nets.REGCN(g, R, 100.0, 64, 64, 3, 2, F.elu, 0.0, [16]).to(DEV).eval()
    feats = [torch.randn(n, 16, device=DEV)]
    labels = torch.randint(0, 3, (n // 2,), device=DEV)
    W, b = net.head()
    out = {}
    for dt in (torch.float32, torch.bfloat16):
        net.zero_grad()
        h = net.embed([f.to(dt) for f in feats], e_feat)
        assert h.dtype == dt
        _, loss = ops.head_ce(h.float(), W, b, labels)
        loss.backward()
        out[dt] = (h.float().detach(), {k: p.grad.clone() for k, p in net.named_parameters()})
    h32, g32 = out[torch.float32]
    h16, g16 = out[torch.bfloat16]
    rel_err = lambda a, b: float((a - b).abs().max()) / max(1e-6, float(b.abs().max()))
    assert rel_err(h16, h32) < 2e-2
    for k in g32:
        assert rel_err(g16[k], g32[k]) < 5e-2, k
