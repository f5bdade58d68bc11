"""Backward hand-off between chained aggregations (regnn_spmm_bwd_next, ops._NextLink): the
consumer y1 = A1(drop(y0)) forms its producer's pre-scaled gradient rows norm0 * g0 and
<g0, y0> / norm0 in its own epilogue, and the producer y0 = norm0 * A0(norm0 * x) gathers them
without a row pass. Outputs and every gradient equal the fp64 masked composition (torch autograd
on the CPU), the hand-off is taken when y0 has no other consumer, and refused (row pass instead)
when autograd sums another gradient into g0 — REGCN layer 1 -> layer 0, layer/REGraphConv.py:73-98."""
import numpy as np
import pytest
import torch

from oracle import regnn_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _graph(n=900, m=12000, R=5, hub=700, seed=3):
    rng = np.random.default_rng(seed)
    src = rng.integers(0, n, m)
    dst = rng.integers(0, n, m)
    dst[:hub] = 11                                    # one row through the chunked path
    src[hub:2 * hub] = 17                             # one long CSC row (transposed gather)
    rel = rng.integers(1, R + 1, m)
    return src, dst, rel, n, R


@pytest.mark.parametrize("dtype,F", [(torch.float32, 64), (torch.bfloat16, 64),
                                     (torch.bfloat16, 128)])
@pytest.mark.parametrize("p", [0.0, 0.5])
@pytest.mark.parametrize("extra", [False, True])
def test_next_handoff_matches_composition(dtype, F, p, extra, monkeypatch):
    from regnn_hip import ops
    from regnn_hip.graph import RelGraph
    taken = []
    orig = ops._NextLink.take

    def spy(self, gy):
        offered = self.handoff is not None
        r = orig(self, gy)
        if offered:
            taken.append(r is not None)
        return r
    monkeypatch.setattr(ops._NextLink, "take", spy)

    src, dst, rel, n, R = _graph()
    rg = RelGraph(src, dst, n, DEV)
    pack = rg.rel_pack(torch.from_numpy(rel).to(DEV), num_rel=R)
    g = torch.Generator().manual_seed(5)
    x = torch.randn(n, F, generator=g).to(dtype)
    tab0, tab1 = torch.rand(R, 1, generator=g) + 0.2, torch.rand(R, 1, generator=g) + 0.2
    n0, n1 = torch.rand(n, generator=g) + 0.5, torch.rand(n, generator=g) + 0.5
    gy = torch.randn(n, F, generator=g).to(dtype)
    w_extra = torch.randn(n, F, generator=g).to(dtype)
    seed = torch.tensor([0x0F1E_2D3C_4B5A_6978], dtype=torch.int64, device=DEV)

    leaves = [t.to(DEV).requires_grad_(True) for t in (x, tab0, n0, tab1, n1)]
    xd, t0, m0, t1, m1 = leaves
    y0 = ops.re_spmm(rg, xd, t0, pack, pre=m0, post=m0)
    y1 = ops.re_spmm(rg, y0, t1, pack, pre=m1, post=m1, dropout=p, drop_seed=seed)
    loss = (y1.float() * gy.to(DEV).float()).sum()
    if extra:                                          # a second consumer of y0
        loss = loss + (y0.float() * w_extra.to(DEV).float()).sum()
    loss.backward()
    assert taken == [not extra]

    L = [t.double().requires_grad_(True) for t in (x, tab0, n0, tab1, n1)]
    X, T0, N0, T1, N1 = L
    ridx, idx = torch.from_numpy(rel - 1), torch.from_numpy(np.stack([dst, src]))
    A0 = torch.sparse_coo_tensor(idx, T0[ridx, 0], (n, n))
    A1 = torch.sparse_coo_tensor(idx, T1[ridx, 0], (n, n))
    Y0 = N0[:, None] * torch.sparse.mm(A0, X * N0[:, None])
    if dtype == torch.bfloat16:
        Y0r = Y0 + (Y0.detach().to(dtype).double() - Y0.detach())   # y0 is stored in bf16
    else:
        Y0r = Y0
    if p:
        keep16 = int(round((1 - p) * 65536))
        mask = torch.from_numpy(O.dropout_mask(int(seed.item()), n, F, 16 // x.element_size(),
                                               keep16))
        Y0d = Y0r * mask / (1 - p)
    else:
        Y0d = Y0r
    Y1 = N1[:, None] * torch.sparse.mm(A1, Y0d * N1[:, None])
    Loss = (Y1 * gy.double()).sum()
    if extra:
        Loss = Loss + (Y0 * w_extra.double()).sum()
    Loss.backward()
    tol = 1e-5 if dtype == torch.float32 else 3e-2
    scale = lambda t: max(1.0, float(t.abs().max()))
    for tag, a, b in (("y1", y1, Y1), ("gx", xd.grad, X.grad), ("gtab0", t0.grad, T0.grad),
                      ("gnorm0", m0.grad, N0.grad), ("gtab1", t1.grad, T1.grad),
                      ("gnorm1", m1.grad, N1.grad)):
        err = float((a.detach().double().cpu() - b.detach()).abs().max()) / scale(b)
        assert err <= tol, f"{tag}: rel err {err:.3e}"


def test_next_handoff_equals_row_pass():
    """the hand-off and the producer's own row pass give the same gradients (fp32, p = 0.5)."""
    from regnn_hip import ops
    from regnn_hip.graph import RelGraph
    src, dst, rel, n, R = _graph(seed=8)
    rg = RelGraph(src, dst, n, DEV)
    pack = rg.rel_pack(torch.from_numpy(rel).to(DEV), num_rel=R)
    g = torch.Generator().manual_seed(2)
    base = [torch.randn(n, 64, generator=g), torch.rand(R, 1, generator=g) + 0.2,
            torch.rand(n, generator=g) + 0.5, torch.rand(R, 1, generator=g) + 0.2,
            torch.rand(n, generator=g) + 0.5]
    gy = torch.randn(n, 64, generator=g).to(DEV)
    seed = torch.tensor([77], dtype=torch.int64, device=DEV)
    grads = {}
    old = dict(ops.PRESCALE)
    try:
        for mode in ("auto", "off"):
            ops.PRESCALE["next"] = mode
            xd, t0, m0, t1, m1 = [t.to(DEV).requires_grad_(True) for t in base]
            y0 = ops.re_spmm(rg, xd, t0, pack, pre=m0, post=m0)
            y1 = ops.re_spmm(rg, y0, t1, pack, pre=m1, post=m1, dropout=0.5, drop_seed=seed)
            y1.backward(gy)
            grads[mode] = [t.grad.clone() for t in (xd, t0, m0, t1, m1)]
    finally:
        ops.PRESCALE.update(old)
    for a, b in zip(grads["auto"], grads["off"]):
        err = float((a - b).abs().max()) / max(1.0, float(b.abs().max()))
        assert err <= 1e-6


@pytest.mark.parametrize("dtype,F", [(torch.float32, 64), (torch.bfloat16, 64),
                                     (torch.bfloat16, 128)])
@pytest.mark.parametrize("p", [0.0, 0.5, 0.75, 0.3])
def test_fwd_emit_equals_row_pass(dtype, F, p):
    """regnn_spmm_fwd_next: the consumer's rows drop(scale * y) from the epilogue are
    bit-identical to regnn_row_scale over the stored y with the same scale and seed."""
    from regnn_hip import ops
    from regnn_hip import _lib as L
    from regnn_hip.graph import RelGraph
    src, dst, rel, n, R = _graph(seed=4)
    rg = RelGraph(src, dst, n, DEV)
    pack = rg.rel_pack(torch.from_numpy(rel).to(DEV), num_rel=R)
    g = torch.Generator().manual_seed(9)
    x = torch.randn(n, F, generator=g).to(dtype).to(DEV)
    tab = (torch.rand(R, 1, generator=g) + 0.2).to(DEV)
    m0 = (torch.rand(n, generator=g) + 0.5).to(DEV)
    s1 = (torch.rand(n, generator=g) + 0.5).to(DEV)
    bias = torch.randn(F, generator=g).to(DEV)
    drop = ops.drop_request(p, DEV, torch.tensor([991], dtype=torch.int64, device=DEV)) \
        if p else None
    with torch.no_grad():
        y, xs = ops.re_spmm(rg, x, tab, pack, pre=m0, post=m0, bias=bias, emit=(s1, drop))
        y_ref = ops.re_spmm(rg, x, tab, pack, pre=m0, post=m0, bias=bias)
        ref = torch.empty_like(y)
        L.call("regnn_row_scale", L.ptr(y), L.ptr(s1), L.ptr(ref), n, F, L.dtype_code(y),
               *(ops._drop_args(drop)), None, None, L.stream())
    assert xs is not None
    assert torch.equal(y, y_ref)
    assert torch.equal(xs, ref)


@pytest.mark.parametrize("train", [False, True])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_regcn_chained_matches_unchained(train, dtype):
    """nets.FUSE_NEXT: REGCN with layer 1's pre-scaled rows from layer 0's epilogue (and the
    backward hand-off) equals the unchained composition: h, loss and every gradient."""
    import torch.nn.functional as F
    from regnn_hip import nets, ops, synth
    import dgl
    gd = synth.mag_like(0.002, seed=3, device=DEV)
    g = dgl.DGLGraph((gd["src"], gd["dst"]), num_nodes=gd["N"])
    e_feat = gd["rel"].to(torch.int64)
    feats = synth.type_features(gd["counts"], {t: 128 for t in synth.NTYPES}, seed=1, device=DEV,
                                kind="mag")
    feats = [f.to(dtype) for f in feats]
    torch.manual_seed(0)
    net = nets.REGCN(g, gd["R"], 100.0, 64, 64, 349, 2, F.elu, 0.5,
                     [f.shape[1] for f in feats]).to(DEV)
    net.train(train)
    labels = torch.randint(0, 349, (gd["counts"]["paper"],), device=DEV)
    W, b = net.head()
    out = {}
    old = (nets.FUSE_NEXT, dict(ops.PRESCALE))
    try:
        for fused in (False, True):
            nets.FUSE_NEXT = fused
            ops.PRESCALE["next"] = "auto" if fused else "off"
            ops._DROP_CTR.clear()
            torch.manual_seed(5)                         # same dropout seeds in both runs
            net.zero_grad()
            h = net.embed(feats, e_feat)
            _, loss = ops.head_ce(h.float(), W, b, labels)
            loss.backward()
            out[fused] = (h.detach().float().clone(), float(loss),
                          {k: p.grad.clone() for k, p in net.named_parameters()
                           if p.grad is not None})
    finally:
        nets.FUSE_NEXT = old[0]
        ops.PRESCALE.update(old[1])
    (h0, l0, g0), (h1, l1, g1) = out[False], out[True]
    rel = lambda a, b: float((a - b).abs().max()) / max(1.0, float(b.abs().max()))
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert rel(h1, h0) <= tol
    assert abs(l1 - l0) <= tol * max(1.0, abs(l0))
    assert g0.keys() == g1.keys()
    for k in g0:
        assert rel(g1[k], g0[k]) <= (1e-4 if dtype == torch.float32 else 2e-2), k


@pytest.mark.parametrize("mode", ["z", "p"])
@pytest.mark.parametrize("n_loss", [20, 333, 900])
def test_head_gh_handoff(n_loss, mode, monkeypatch):
    """regnn_head_gh_next / regnn_head_bwd_z: the output head's gh kernel forms the last
    aggregation's pre-scaled gradient rows (zero rows without a loss term); gradients equal the
    row-pass path, with p stored (p) or re-formed from the logits rows (z)."""
    from regnn_hip import ops
    monkeypatch.setitem(ops.HEAD, "p", mode)
    from regnn_hip.graph import RelGraph
    taken = []
    orig = ops._NextLink.take

    def spy(self, gy):
        offered = self.handoff is not None
        r = orig(self, gy)
        if offered:
            taken.append(r is not None)
        return r
    monkeypatch.setattr(ops._NextLink, "take", spy)
    src, dst, rel, n, R = _graph(seed=6)
    rg = RelGraph(src, dst, n, DEV)
    pack = rg.rel_pack(torch.from_numpy(rel).to(DEV), num_rel=R)
    g = torch.Generator().manual_seed(4)
    C = 37
    base = [torch.randn(n, 64, generator=g), torch.rand(R, 1, generator=g) + 0.2,
            torch.rand(n, generator=g) + 0.5, torch.randn(C, 64, generator=g) * 0.1,
            torch.randn(C, generator=g)]
    labels = torch.randint(0, C, (n_loss,), generator=g).to(DEV)
    grads = {}
    old = dict(ops.PRESCALE)
    try:
        for mode in ("auto", "noprefix", "off"):
            ops.PRESCALE["next"] = "off" if mode == "off" else "auto"
            ops.PRESCALE["prefix"] = "off" if mode == "noprefix" else "auto"
            taken.clear()
            xd, t0, m0, W, b = [t.to(DEV).requires_grad_(True) for t in base]
            y = ops.re_spmm(rg, xd, t0, pack, pre=m0, post=m0)
            _, loss = ops.head_ce(y, W, b, labels)
            loss.backward()
            # (without the prefix, the producer declines a truncating hand-off after taking it)
            assert taken == ([True] if mode != "off" else [])
            grads[mode] = [t.grad.clone() for t in (xd, t0, m0, W, b)]
    finally:
        ops.PRESCALE.update(old)
    # the CSC prefix (edges into loss rows only) changes the long rows' chunking: rounding only
    for m in ("auto", "noprefix"):
        for a, b in zip(grads[m], grads["off"]):
            err = float((a - b).abs().max()) / max(1.0, float(b.abs().max()))
            assert err <= 1e-6


@pytest.mark.parametrize("n_loss", [20, 333])
def test_head_gh_handoff_bf16(n_loss, monkeypatch):
    """bf16 feature pipeline: head_ce takes the aggregation's bf16 rows, its z-mode gh kernel
    stores the bf16 gradient and the producer's bf16 pre-scaled rows (regnn_head_bwd_z dtype 1);
    gradients match the unlinked path (bf16 gradient from the head, row pass in the producer)."""
    from regnn_hip import ops
    from regnn_hip.graph import RelGraph
    monkeypatch.setitem(ops.HEAD, "p", "z")
    taken = []
    orig = ops._NextLink.take

    def spy(self, gy):
        offered = self.handoff is not None
        r = orig(self, gy)
        if offered:
            taken.append(r is not None)
        return r
    monkeypatch.setattr(ops._NextLink, "take", spy)
    src, dst, rel, n, R = _graph(seed=8)
    rg = RelGraph(src, dst, n, DEV)
    pack = rg.rel_pack(torch.from_numpy(rel).to(DEV), num_rel=R)
    g = torch.Generator().manual_seed(5)
    C = 349
    base = [torch.randn(n, 64, generator=g), torch.rand(R, 1, generator=g) + 0.2,
            torch.rand(n, generator=g) + 0.5, torch.randn(C, 64, generator=g) * 0.1,
            torch.randn(C, generator=g)]
    labels = torch.randint(0, C, (n_loss,), generator=g).to(DEV)
    grads, losses = {}, {}
    old = dict(ops.PRESCALE)
    try:
        for mode in ("auto", "noprefix", "off"):
            ops.PRESCALE["next"] = "off" if mode == "off" else "auto"
            ops.PRESCALE["prefix"] = "off" if mode == "noprefix" else "auto"
            taken.clear()
            xd, t0, m0, W, b = [t.to(DEV).requires_grad_(True) for t in base]
            y = ops.re_spmm(rg, xd.bfloat16(), t0, pack, pre=m0, post=m0)
            assert y.dtype == torch.bfloat16
            _, loss = ops.head_ce(y, W, b, labels)
            loss.backward()
            # (without the prefix, the producer declines a truncating hand-off after taking it)
            assert taken == ([True] if mode != "off" else [])
            grads[mode] = [t.grad.clone() for t in (xd, t0, m0, W, b)]
            losses[mode] = loss.item()
    finally:
        ops.PRESCALE.update(old)
    assert losses["auto"] == losses["off"]
    for m in ("auto", "noprefix"):
        for a, b in zip(grads[m], grads["off"]):
            err = float((a - b).abs().max()) / max(1e-3, float(b.abs().max()))
            assert err <= 1e-2


@pytest.mark.parametrize("n_loss", [20, 333])
def test_head_ce_non_prefix_loss_rows(n_loss):
    """head_ce with an arbitrary loss-row set (rows=): loss and every gradient equal torch's
    cross-entropy over logits[rows] (run_regnn.py:146-148 with a random train split)."""
    from regnn_hip import ops
    from regnn_hip.graph import RelGraph
    src, dst, rel, n, R = _graph(seed=9)
    rg = RelGraph(src, dst, n, DEV)
    pack = rg.rel_pack(torch.from_numpy(rel).to(DEV), num_rel=R)
    g = torch.Generator().manual_seed(6)
    C = 37
    base = [torch.randn(n, 64, generator=g), torch.rand(R, 1, generator=g) + 0.2,
            torch.rand(n, generator=g) + 0.5, torch.randn(C, 64, generator=g) * 0.1,
            torch.randn(C, generator=g)]
    rows = torch.randperm(n, generator=g)[:n_loss].to(DEV)
    labels = torch.randint(0, C, (n_loss,), generator=g).to(DEV)
    out = []
    for fused in (True, False):
        xd, t0, m0, W, b = [t.to(DEV).requires_grad_(True) for t in base]
        y = ops.re_spmm(rg, xd, t0, pack, pre=m0, post=m0)
        if fused:
            logits, loss = ops.head_ce(y, W, b, labels, rows=rows)
        else:
            logits = y @ W.t() + b
            loss = torch.nn.functional.cross_entropy(logits[rows], labels)
        loss.backward()
        out.append([loss.detach(), logits.detach()] + [t.grad for t in (xd, t0, m0, W, b)])
    for name, a, b_ in zip(["loss", "logits", "x", "tab", "scale", "W", "b"], out[0], out[1]):
        err = (a - b_).abs().max().item() / max(1.0, b_.abs().max().item())
        assert err <= 1e-5, f"{name}: rel err {err:.3e}"


def test_loss_rows_first_renumbering_preserves_the_model():
    """data.loss_rows_first: REGCN on the renumbered graph with head_ce's prefix fast path gives
    the loss and parameter gradients of the original numbering with the loss over a random
    (non-prefix) train split."""
    import torch.nn.functional as F
    import dgl
    from regnn_hip import data, nets, ops, synth
    gd = synth.mag_like(0.002, seed=3, device=DEV)
    feats = synth.type_features(gd["counts"], {t: 16 for t in synth.NTYPES}, seed=1, device=DEV)
    n_paper = gd["counts"]["paper"]
    gen = torch.Generator(device=DEV).manual_seed(2)
    train = torch.randperm(n_paper, generator=gen, device=DEV)[:n_paper // 2]
    y = torch.randint(0, 7, (n_paper,), generator=gen, device=DEV)
    res = []
    for renumber in (False, True):
        src, dst, fs = gd["src"], gd["dst"], list(feats)
        lab_rows, lab = train, y[train]
        if renumber:
            perm, inv = data.loss_rows_first(gd["N"], train, n_paper)
            src, dst = inv[src], inv[dst]
            fs[0] = fs[0][perm[:n_paper]].contiguous()
            lab = y[perm[:train.numel()]]
        g = dgl.DGLGraph((src, dst), num_nodes=gd["N"])
        torch.manual_seed(0)
        net = nets.REGCN(g, gd["R"], 100.0, 64, 64, 7, 2, F.elu, 0.0,
                         [f.shape[1] for f in fs]).to(DEV).eval()
        h = net.embed(fs, gd["rel"].to(torch.int64))
        W, b = net.head()
        if renumber:
            _, loss = ops.head_ce(h, W, b, lab)
        else:
            loss = F.cross_entropy((h @ W.t() + b)[lab_rows], lab)
        loss.backward()
        res.append((loss.detach(), {n: p.grad.clone() for n, p in net.named_parameters()}))
    (l0, g0), (l1, g1) = res
    assert abs(float(l0) - float(l1)) <= 1e-5 * max(1.0, abs(float(l0)))
    for k in g0:
        err = (g0[k] - g1[k]).abs().max().item() / max(1.0, g0[k].abs().max().item())
        assert err <= 1e-5, f"{k}: rel err {err:.3e}"
