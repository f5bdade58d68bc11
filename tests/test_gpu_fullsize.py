"""Parity at the BASELINE full size (mag_like(10): N = 19.4 M, E = 441.6 M, R = 11, F = 64 fp32,
the graph bench.py measures), through properties that do not need an O(E) CPU oracle run:

* sampled rows (random rows + the largest hubs, i.e. the chunk + tree path) of the forward
  aggregation and of the transposed backward aggregation against fp64 sums over the CSR / CSC
  rows computed on the device (layer/REGraphConv.py:66-101 composition: norm pre-scale, relation
  table, norm post-scale);
* the weighted degree: sampled rows, and sum(deg) = sum_r tab[r] * count_r (a checksum over all
  441 M edges);
* adjointness of forward and backward, <A x, g> = <x, A^T g>, over every element;
* linearity in the relation table: d<y, g>/d tab[r] (the fused relation-bin gradient) equals
  <A_{e_r} x, g>, the forward run with the one-hot table e_r, for every relation r.
"""
import os
import sys
import time

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
F = 64
SCALE = float(os.environ.get("REGNN_FULLSIZE_SCALE", "10"))   # 10 = BASELINE mag-10x
_T0 = time.time()


def _log(msg):
    torch.cuda.synchronize()
    print(f"[fullsize +{time.time() - _T0:.1f}s] {msg}", file=sys.stderr, flush=True)


@pytest.fixture(scope="module")
def big():
    from regnn_hip import ops, synth
    from regnn_hip.graph import RelGraph
    _log(f"building mag_like({SCALE})")
    gd = synth.mag_like(SCALE, seed=0, device=DEV)
    R = gd["R"]
    rg = RelGraph(gd["src"], gd["dst"], gd["N"], DEV)
    rel = gd["rel"].to(torch.int64)
    pack = rg.rel_pack(rel, R)
    counts = torch.bincount(rel - 1, minlength=R).to(torch.float64)
    del gd
    _log(f"graph N={rg.n_dst:,} E={rg.E:,}")
    g = torch.Generator(device=DEV)
    g.manual_seed(7)
    # alpha * w ~ U(-0.5, 1.5): both LeakyReLU slopes, some weighted degrees below 1 (clamp)
    tab = torch.nn.functional.leaky_relu(torch.rand(R, 1, generator=g, device=DEV) * 2 - 0.5)
    x = torch.randn(rg.n_src, F, generator=g, device=DEV)
    gy = torch.randn(rg.n_dst, F, generator=g, device=DEV)
    with torch.no_grad():
        norm = ops.degree_norm(rg, pack, tab)
    _log("inputs ready")
    yield dict(rg=rg, pack=pack, tab=tab, x=x, gy=gy, norm=norm, counts=counts, R=R)
    torch.cuda.empty_cache()


def _rows(rg, n_random=3000, n_hubs=8, seed=3):
    deg = rg.csr_ptr[1:] - rg.csr_ptr[:-1]
    hubs = torch.topk(deg, n_hubs).indices
    g = torch.Generator(device=DEV)
    g.manual_seed(seed)
    rnd = torch.randint(0, rg.n_dst, (n_random,), generator=g, device=DEV)
    return torch.unique(torch.cat([hubs, rnd]))


def _segment_sums(ptr, idx, rel, rows, val_fn, chunk=1 << 22, big=4096):
    """fp64 sums over the segments `rows` of val_fn(neighbour ids, rel ids) -> [len(rows), ...].
    Segments longer than `big` (the hubs, ~11 M edges) are reduced chunk by chunk with plain sums;
    the rest through one index_add_ (a scatter into a few hub rows would serialise on fp64
    atomics)."""
    b = ptr[rows].to(torch.int64)
    e = ptr[rows + 1].to(torch.int64)
    cnt = e - b
    out = None
    for k in torch.nonzero(cnt > big).flatten().tolist():
        acc = None
        for s in range(int(b[k]), int(e[k]), chunk):
            sl = slice(s, min(int(e[k]), s + chunk))
            part = val_fn(idx[sl].to(torch.int64), rel[sl].to(torch.int64)).sum(0)
            acc = part if acc is None else acc + part
        if out is None:
            out = torch.zeros((rows.numel(),) + tuple(acc.shape), dtype=torch.float64, device=DEV)
        out[k] = acc
    small = torch.nonzero(cnt <= big).flatten()
    cs = cnt[small]
    seg = torch.repeat_interleave(small, cs)
    pos = torch.arange(seg.numel(), device=DEV) - (torch.cumsum(cs, 0) - cs).repeat_interleave(cs) \
        + b[small].repeat_interleave(cs)
    vals = val_fn(idx[pos].to(torch.int64), rel[pos].to(torch.int64))
    if out is None:
        out = torch.zeros((rows.numel(),) + tuple(vals.shape[1:]), dtype=torch.float64, device=DEV)
    out.index_add_(0, seg, vals)
    return out


def _close(got, want, tol=1e-5):
    err = float((got.double() - want).abs().max()) / max(1.0, float(want.abs().max()))
    return err <= tol, err


def test_fullsize_degree(big):
    rg, pack, tab, counts = big["rg"], big["pack"], big["tab"], big["counts"]
    from regnn_hip import ops
    norm, deg = ops._DegreeNorm.apply(tab, rg, pack, -0.5)
    want_total = float((tab.double().reshape(-1) * counts).sum())
    got_total = float(deg.double().sum())
    assert abs(got_total - want_total) <= 1e-6 * abs(want_total)
    rows = _rows(rg)
    t64 = tab.double().reshape(-1)
    want = _segment_sums(rg.csr_ptr, rg.csr_idx, pack.rel_csr, rows, lambda u, r: t64[r])
    ok, err = _close(deg[rows], want, 1e-5)
    assert ok, f"sampled degrees: {err:.3e}"
    ok, err = _close(norm[rows], want.clamp(min=1).pow(-0.5), 1e-5)
    assert ok, f"sampled norms: {err:.3e}"
    _log("degree checked")


def test_fullsize_forward_backward_rows(big):
    from regnn_hip import ops
    rg, pack, tab, x, gy, norm = (big[k] for k in ("rg", "pack", "tab", "x", "gy", "norm"))
    t64, n64 = tab.double().reshape(-1), norm.double()
    xr = x.clone().requires_grad_(True)
    y = ops.re_spmm(rg, xr, tab, pack, pre=norm, post=norm)
    y.backward(gy)
    _log("fwd + bwd done")
    rows = _rows(rg)
    want = _segment_sums(rg.csr_ptr, rg.csr_idx, pack.rel_csr, rows,
                         lambda u, r: (t64[r] * n64[u])[:, None] * x[u].double())
    want *= n64[rows][:, None]
    ok, err = _close(y[rows].detach(), want)
    assert ok, f"forward rows (hubs included): {err:.3e}"
    _log("forward rows checked")
    cols = _rows(rg, seed=5)
    want = _segment_sums(rg.csc_ptr, rg.csc_idx, pack.rel_csc, cols,
                         lambda v, r: (t64[r] * n64[v])[:, None] * gy[v].double())
    want *= n64[cols][:, None]
    ok, err = _close(xr.grad[cols], want)
    assert ok, f"backward rows (hubs included): {err:.3e}"
    # adjointness over every element: <A x, g> = <x, A^T g>
    lhs = float((y.detach().double() * gy.double()).sum())
    rhs = float((x.double() * xr.grad.double()).sum())
    assert abs(lhs - rhs) <= 1e-5 * max(abs(lhs), abs(rhs)) + 1e-3, (lhs, rhs)


def test_fullsize_relation_gradient_linearity(big):
    from regnn_hip import ops
    rg, pack, tab, x, gy, norm, R = (big[k] for k in ("rg", "pack", "tab", "x", "gy", "norm", "R"))
    t = tab.clone().requires_grad_(True)
    y = ops.re_spmm(rg, x, t, pack, pre=norm, post=norm)        # norm fixed: y linear in t
    y.backward(gy)
    got = t.grad.double().reshape(-1)
    with torch.no_grad():
        for r in range(R):
            onehot = torch.zeros_like(tab)
            onehot[r] = 1.0
            yr = ops.re_spmm(rg, x, onehot, pack, pre=norm, post=norm)
            prod = yr.double() * gy.double()
            want, mag = float(prod.sum()), float(prod.abs().sum())
            _log(f"relation {r}: {float(got[r]):.6e} vs {want:.6e} (sum |terms| {mag:.3e})")
            # fp32 accumulation of ~1e8 signed terms: bound the error by their magnitude, not by
            # the (cancelling) sum
            assert abs(float(got[r]) - want) <= 1e-6 * mag + 1e-5 * abs(want), \
                (r, float(got[r]), want, mag)
