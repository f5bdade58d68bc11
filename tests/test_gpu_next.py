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
