"""Per-node-type input rows of the ogbn-mag path (mag/regnn_ns.py:300-326, REGNN.group_input):
regnn_typed_linear_fwd / _wgrad (per-type Linear fused with the gather, fp32 MFMA) and
regnn_typed_gather / _scatter (feats_type 2's table rows and their gradient) against an fp64
restatement of the reference's per-type mask loop; deterministic reruns; edge cases (a type with
no rows, a type without a table, one row, shared weight groups)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _batch(counts, n_pick, seed=0):
    """global node ids type-contiguous per type (counts rows each), a shuffled n_id subset."""
    g = torch.Generator().manual_seed(seed)
    ntype = torch.cat([torch.full((c,), t, dtype=torch.int64) for t, c in enumerate(counts)])
    local = torch.cat([torch.arange(c, dtype=torch.int64) for c in counts])
    n_id = torch.randperm(ntype.numel(), generator=g)[:n_pick]
    return ntype.to(DEV), local.to(DEV), n_id.to(DEV)


def _ref_linear(tabs, Ws, bs, wg, ntype, local, n_id):
    """regnn_ns.py:316-324: h[mask] = lins[key](x[local[mask]]) per type, in fp64."""
    nt, li = ntype[n_id].cpu(), local[n_id].cpu()
    O = Ws[0].shape[0]
    h = torch.zeros(n_id.numel(), O, dtype=torch.float64)
    for t, x in enumerate(tabs):
        m = nt == t
        W, b = Ws[wg[t]].detach().cpu().double(), bs[wg[t]].detach().cpu().double()
        h[m] = x.cpu().double()[li[m]] @ W.T + b
    return h


def _close(a, b, tol, scale=None):
    """max |a - b| within tol of max(1, max |b|), or of `scale` (the largest sum of |terms|, for
    sums that cancel)."""
    a, b = a.detach().cpu().double(), b.detach().cpu().double()
    ref = max(1.0, b.abs().max().item()) if scale is None else scale
    err = (a - b).abs().max().item() / ref
    assert err <= tol, f"rel err {err:.3e} > {tol}"


@pytest.mark.parametrize("K,O,counts,n_pick", [
    (64, 64, [300, 500, 7, 90], 700),
    (128, 64, [1000, 1500, 0, 400], 2500),        # a type with no rows at all
    (128, 512, [2000, 3000, 40, 600], 4000),       # the reference's default width 512
    (256, 128, [50, 60, 70, 80], 255),
    (128, 64, [1, 0, 0, 0], 1),                    # one row
])
def test_typed_linear_vs_fp64(K, O, counts, n_pick):
    from regnn_hip import ops
    torch.manual_seed(K + O)
    ntype, local, n_id = _batch(counts, n_pick, seed=K)
    tabs = [torch.randn(max(c, 1), K, device=DEV) for c in counts]
    Ws = [torch.randn(O, K, device=DEV, requires_grad=True) for _ in counts]
    bs = [torch.randn(O, device=DEV, requires_grad=True) for _ in counts]
    y = ops.typed_linear(tabs, Ws, bs, ntype, local, n_id)
    ref = _ref_linear(tabs, Ws, bs, list(range(4)), ntype, local, n_id)
    _close(y, ref, 1e-5)
    gy = torch.randn_like(y)
    y.backward(gy)
    nt, li = ntype[n_id].cpu(), local[n_id].cpu()
    for t in range(4):
        m = nt == t
        X = tabs[t].cpu().double()[li[m]]
        G = gy.cpu().double()[m]
        _close(Ws[t].grad, G.T @ X, 1e-5)
        _close(bs[t].grad, G.sum(0), 1e-5)


def test_typed_linear_shared_weight_and_determinism():
    """wgroup: every type through one Linear (the gradient summed over all types' runs in
    fixed chunk order); two runs bitwise equal."""
    from regnn_hip import ops
    torch.manual_seed(3)
    counts = [3000, 2500, 100, 1200]
    ntype, local, n_id = _batch(counts, 6000, seed=5)
    tabs = [torch.randn(c, 128, device=DEV) for c in counts]
    W = torch.randn(64, 128, device=DEV, requires_grad=True)
    b = torch.randn(64, device=DEV, requires_grad=True)
    outs = []
    for _ in range(2):
        W.grad = b.grad = None
        y = ops.typed_linear(tabs, [W], [b], ntype, local, n_id, wgroup=[0, 0, 0, 0])
        gy = torch.sin(torch.arange(y.numel(), device=DEV, dtype=torch.float32)).view_as(y)
        y.backward(gy)
        outs.append((y.detach().clone(), W.grad.clone(), b.grad.clone()))
    for a, c in zip(outs[0], outs[1]):
        assert torch.equal(a, c)
    ref = _ref_linear(tabs, [W], [b], [0, 0, 0, 0], ntype, local, n_id)
    _close(outs[0][0], ref, 1e-5)
    nt, li = ntype[n_id].cpu(), local[n_id].cpu()
    X = torch.zeros(n_id.numel(), 128, dtype=torch.float64)
    for t in range(4):
        X[nt == t] = tabs[t].cpu().double()[li[nt == t]]
    G = gy.cpu().double()
    _close(outs[0][1], G.T @ X, 1e-5)
    _close(outs[0][2], G.sum(0), 1e-6, scale=G.abs().sum(0).max().item())


def test_typed_gather_scatter():
    """feats_type 2's input matrix (regnn_ns.py:307-314): target rows from the raw features,
    the others from learned tables, a type without a table -> zero rows; the backward adds
    each row's gradient into its table row (and nowhere else)."""
    from regnn_hip import ops
    torch.manual_seed(4)
    counts = [400, 300, 200, 100]
    ntype, local, n_id = _batch(counts, 800, seed=7)
    x0 = torch.randn(400, 32, device=DEV)
    e1 = torch.randn(300, 32, device=DEV, requires_grad=True)
    e2 = torch.randn(200, 32, device=DEV, requires_grad=True)
    out = ops.typed_gather([x0, e1, e2, None], ntype, local, n_id)
    nt, li = ntype[n_id].cpu(), local[n_id].cpu()
    ref = torch.zeros(800, 32)
    ref[nt == 0] = x0.cpu()[li[nt == 0]]
    ref[nt == 1] = e1.detach().cpu()[li[nt == 1]]
    ref[nt == 2] = e2.detach().cpu()[li[nt == 2]]
    assert torch.equal(out.cpu(), ref)
    g = torch.randn_like(out)
    out.backward(g)
    for t, e in ((1, e1), (2, e2)):
        want = torch.zeros_like(e.detach().cpu())
        want[li[nt == t]] = g.cpu()[nt == t]
        assert torch.equal(e.grad.cpu(), want)


def test_group_input_ft3_typed_matches_all_types_gemm():
    """mag.REGNN.group_input (feats_type 3, 128-d inputs, hidden 512: the reference defaults)
    through the typed launch equals the per-type mask loop, and so do the lins gradients."""
    from regnn_hip import mag
    torch.manual_seed(6)
    counts = [5000, 7000, 300, 900]
    ntype, local, n_id = _batch(counts, 9000, seed=9)
    x_dict = {t: torch.rand(c, 128, device=DEV) - 0.5 for t, c in enumerate(counts)}
    net = mag.REGNN(128, 512, 349, 2, 10.0, 0.0, {k: 128 for k in range(4)}, 7,
                    use_norm="ln", self_loop_type=2).to(DEV)
    h = net.group_input(x_dict, ntype, local, n_id)
    Ws = [net.lins[str(t)].weight for t in range(4)]
    bs = [net.lins[str(t)].bias for t in range(4)]
    ref = _ref_linear([x_dict[t] for t in range(4)], Ws, bs, list(range(4)), ntype, local, n_id)
    _close(h, ref, 1e-5)
    gy = torch.randn_like(h)
    h.backward(gy)
    nt, li = ntype[n_id].cpu(), local[n_id].cpu()
    for t in range(4):
        m = nt == t
        _close(Ws[t].grad, gy.cpu().double()[m].T @ x_dict[t].cpu().double()[li[m]], 1e-5)
        _close(bs[t].grad, gy.cpu().double()[m].sum(0), 1e-5)
