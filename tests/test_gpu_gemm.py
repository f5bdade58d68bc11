"""regnn_gemm_x6 (bf16x6: fp32 operands split into three bf16 parts, six MFMA products in fp32)
against fp64 products: every layout, ragged M / N / K tails, split-K, beta accumulation, and the
autograd wrapper's gradients. Tolerance: 2e-6 x sum_k |a_mk b_kn| (fp32 accumulation over K)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ref(a, b, ta, tb):
    a64, b64 = a.double(), b.double()
    A = a64.t() if ta else a64
    B = b64.t() if tb else b64
    return A @ B, A.abs() @ B.abs()


@pytest.mark.parametrize("ta,tb", [(False, False), (False, True), (True, False), (True, True)])
@pytest.mark.parametrize("M,N,K", [(5606, 512, 512), (100, 68, 36), (512, 512, 13312),
                                   (64, 64, 32), (1, 4, 4), (333, 132, 1000),
                                   (512, 349, 512), (349, 512, 512), (13312, 4, 512),
                                   (4, 512, 13312)])
def test_gemm_x6_layouts(ta, tb, M, N, K):
    from regnn_hip import ops
    g = torch.Generator(device=DEV).manual_seed(M + 7 * N + 13 * K)
    a = torch.randn(*((K, M) if ta else (M, K)), generator=g, device=DEV)
    b = torch.randn(*((N, K) if tb else (K, N)), generator=g, device=DEV)
    if not (ops.gemm_x6_ok(a) and ops.gemm_x6_ok(b)):
        pytest.skip("contiguous dimension not a multiple of 4")
    c = ops.gemm_x6(a, b, trans_a=ta, trans_b=tb)
    ref, mag = _ref(a, b, ta, tb)
    err = (c.double() - ref).abs()
    assert (err <= 2e-6 * mag + 1e-30).all(), float((err / (mag + 1e-30)).max())


def test_gemm_x6_beta_and_splits_deterministic():
    from regnn_hip import ops
    g = torch.Generator(device=DEV).manual_seed(3)
    a = torch.randn(13312, 256, generator=g, device=DEV)
    b = torch.randn(13312, 128, generator=g, device=DEV)
    c0 = torch.randn(256, 128, generator=g, device=DEV)
    assert ops._gemm_splits(256, 128, 13312) > 1
    outs = []
    for _ in range(2):
        c = c0.clone()
        ops.gemm_x6(a, b, trans_a=True, out=c, beta=1.0)
        outs.append(c)
    assert torch.equal(outs[0], outs[1])
    ref = c0.double() + a.double().t() @ b.double()
    mag = c0.double().abs() + a.double().abs().t() @ b.double().abs()
    assert ((outs[0].double() - ref).abs() <= 2e-6 * mag).all()


def test_mm_autograd_matches_fp64():
    from regnn_hip import ops
    g = torch.Generator(device=DEV).manual_seed(5)
    a = torch.randn(777, 256, generator=g, device=DEV, requires_grad=True)
    b = torch.randn(256, 512, generator=g, device=DEV, requires_grad=True)
    bias = torch.randn(512, generator=g, device=DEV, requires_grad=True)
    gout = torch.randn(777, 512, generator=g, device=DEV)
    y = ops.mm(a, b, bias)
    y.backward(gout)
    a64, b64, c64 = (t.detach().double().requires_grad_() for t in (a, b, bias))
    y64 = c64 + a64 @ b64
    y64.backward(gout.double())
    for got, want in ((y, y64), (a.grad, a64.grad), (b.grad, b64.grad), (bias.grad, c64.grad)):
        scale = max(1.0, float(want.abs().max()))
        assert float((got.double() - want).abs().max()) <= 1e-5 * scale


@pytest.mark.parametrize("H,dropout,res", [(512, 0.5, True), (128, 0.0, False), (1024, 0.3, False),
                                           (64, 0.5, True)])
def test_wide_ln_act_matches_autograd(H, dropout, res):
    """ops.wide_ln_act (regnn_wide_ln_fwd / _bwd) against torch autograd of rs x + bias + res ->
    LayerNorm -> relu -> (the same hash mask) in fp64: output and every input gradient."""
    from oracle import regnn_oracle as O
    from regnn_hip import ops
    import test_gpu_ns_engine as E
    g = torch.Generator(device=DEV).manual_seed(H)
    n = 1000
    x = torch.randn(n, H, generator=g, device=DEV, requires_grad=True)
    rs = torch.rand(n, generator=g, device=DEV) + 0.5
    bias = torch.randn(H, generator=g, device=DEV, requires_grad=True)
    r = torch.randn(n, H, generator=g, device=DEV, requires_grad=True) if res else None
    ln = torch.nn.LayerNorm(H).to(DEV)
    with torch.no_grad():
        ln.weight.normal_(1, 0.2)
        ln.bias.normal_(0, 0.2)
    state = torch.tensor([123, 2, 0, 9, 0, 0, 0, 0], dtype=torch.int64, device=DEV)
    gy = torch.randn(n, H, generator=g, device=DEV)
    y = ops.wide_ln_act(x, bias, ln, dropout, state, 1, rs=rs, res=r)
    y.backward(gy)
    keep16 = int(round((1 - dropout) * 65536))
    mask = torch.from_numpy(O.dropout_mask(E._nsm_seed(state.cpu().tolist(), 1), n, H, 4, keep16)
                            ).to(DEV) / (keep16 / 65536) if dropout > 0 else 1.0
    x64, b64 = x.detach().double().requires_grad_(), bias.detach().double().requires_grad_()
    w64, lb64 = ln.weight.detach().double().requires_grad_(), ln.bias.detach().double().requires_grad_()
    r64 = r.detach().double().requires_grad_() if res else None
    a = rs.double()[:, None] * x64 + b64 + (r64 if res else 0)
    y64 = torch.relu(torch.nn.functional.layer_norm(a, (H,), w64, lb64, 1e-5)) * mask
    y64.backward(gy.double())
    pairs = [(y, y64), (x.grad, x64.grad), (bias.grad, b64.grad), (ln.weight.grad, w64.grad),
             (ln.bias.grad, lb64.grad)] + ([(r.grad, r64.grad)] if res else [])
    for got, want in pairs:
        scale = max(1.0, float(want.abs().max()))
        assert float((got.double() - want).abs().max()) <= 2e-5 * scale


def test_linear_x6_autograd_matches_fp64():
    """ops.linear (out_lin: 349 classes, rows of 349 floats load per element) forward and
    backward against fp64."""
    from regnn_hip import ops
    g = torch.Generator(device=DEV).manual_seed(9)
    x = torch.randn(512, 512, generator=g, device=DEV, requires_grad=True)
    w = torch.randn(349, 512, generator=g, device=DEV, requires_grad=True)
    bias = torch.randn(349, generator=g, device=DEV, requires_grad=True)
    gout = torch.randn(512, 349, generator=g, device=DEV)
    y = ops.linear(x, w, bias)
    y.backward(gout)
    x64, w64, g64 = x.detach().double(), w.detach().double(), gout.double()
    checks = [(y, x64 @ w64.t() + bias.detach().double(), x64.abs() @ w64.abs().t()),
              (x.grad, g64 @ w64, g64.abs() @ w64.abs()),
              (w.grad, g64.t() @ x64, g64.abs().t() @ x64.abs())]
    for got, ref, mag in checks:
        err = (got.detach().double() - ref).abs()
        assert (err <= 2e-6 * mag + 1e-6).all(), float((err / (mag + 1e-30)).max())
    assert torch.allclose(bias.grad.double(), g64.sum(0), rtol=1e-5, atol=1e-5)


def test_copy_many_strided_sources():
    """ops.copy_many: one launch copying 2-D (some transposed), 1-D and 0-D sources into
    contiguous destinations, bitwise."""
    from regnn_hip import ops
    g = torch.Generator(device=DEV).manual_seed(1)
    srcs = [torch.randn(128, 512, generator=g, device=DEV).t(),
            torch.randn(512, 512, generator=g, device=DEV),
            torch.randn(349, generator=g, device=DEV),
            torch.randn(64, 4, generator=g, device=DEV)[:, 1],
            torch.randn((), device=DEV)]
    srcs += [torch.randn(3, 5, generator=g, device=DEV) for _ in range(40)]   # > 32: 2 launches
    dsts = [torch.full(tuple(s_.shape), float("nan"), device=DEV) for s_ in srcs]
    ops.copy_many(dsts, srcs)
    for d, s_ in zip(dsts, srcs):
        assert torch.equal(d, s_)


@pytest.mark.parametrize("hint", [None, 6100])
@pytest.mark.parametrize("live", [0, 1, 127, 128, 5606, 13312])
def test_mm_live_rows_bitwise(live, hint, monkeypatch):
    """ops.mm with a live-row count (the capacity-sized block's rows past it are zero): the
    forward and both gradients bitwise those of the full GEMMs on the same zero-padded operands
    (the skipped products are exact zeros), the output's dead rows equal to c's. hint: the
    trainer's typical live rows for this capacity (ops.LIVE_HINT): the 13312-row products split
    K in two (the dead row tiles write no partial, the reduce skips their rows) with and without
    the live count alike; against fp64 at 1e-5 too."""
    from regnn_hip import ops
    monkeypatch.setattr(ops, "LIVE_HINT", {} if hint is None else {13312: hint})
    if hint is not None:
        assert ops._gemm_splits(13312, 512, 516) == 2
    g = torch.Generator(device=DEV).manual_seed(11)
    M, K, N = 13312, 516, 512
    a0 = torch.randn(M, K, generator=g, device=DEV)
    a0[live:] = 0
    b0 = torch.randn(K, N, generator=g, device=DEV)
    c0 = torch.randn(N, generator=g, device=DEV)
    gout = torch.randn(M, N, generator=g, device=DEV)
    gout[live:] = 0
    cnt = torch.tensor([live], dtype=torch.int32, device=DEV)
    outs = []
    for lv in (None, cnt):
        a, b, c = (t.clone().requires_grad_(True) for t in (a0, b0, c0))
        y = ops.mm(a, b, c, live=lv)
        y.backward(gout)
        outs.append([y.detach(), a.grad, b.grad, c.grad])
    for name, x, y in zip(["out", "g_a", "g_b", "g_c"], outs[0], outs[1]):
        assert torch.equal(x, y), name
    ref = c0.double() + a0.double() @ b0.double()
    err = (outs[1][0].double() - ref).abs().max().item() / max(1.0, ref.abs().max().item())
    assert err <= 1e-5, err
    ga = gout.double() @ b0.double().t()
    err = (outs[1][1].double() - ga).abs().max().item() / max(1.0, ga.abs().max().item())
    assert err <= 1e-5, err


@pytest.mark.parametrize("ta,tb", [(False, False), (False, True), (True, False), (True, True)])
@pytest.mark.parametrize("M,N,K,live", [(13312, 512, 516, 4900), (13312, 516, 512, 4900),
                                        (333, 132, 100, 333), (65, 4, 36, 40), (64, 512, 32, 1),
                                        (200, 349, 512, 129)])
def test_gemm_x6_row_tilings_bitwise(ta, tb, M, N, K, live, monkeypatch):
    """a product with a live-row count runs on 64-row tiles (REGNN_GEMM_BM64, no split-K), every
    other on 128-row tiles: each C element sums the same k-steps and products in the same order,
    so the two tilings give the same bits (rows past the live count: beta C either way)."""
    from regnn_hip import ops
    g = torch.Generator(device=DEV).manual_seed(M + 3 * N + 5 * K + live)
    a = torch.randn(*((K, M) if ta else (M, K)), generator=g, device=DEV)
    b = torch.randn(*((N, K) if tb else (K, N)), generator=g, device=DEV)
    if ta:
        a[:, live:] = 0
    else:
        a[live:] = 0
    if not (ops.gemm_x6_ok(a) and ops.gemm_x6_ok(b)):
        pytest.skip("contiguous dimension not a multiple of 4")
    monkeypatch.setattr(ops, "_gemm_splits", lambda *_: 1)
    cnt = torch.tensor([live], dtype=torch.int32, device=DEV)
    outs = {}
    for mode in ("on", "off"):
        monkeypatch.setenv("REGNN_GEMM_BM64", mode)
        outs[mode] = ops.gemm_x6(a, b, trans_a=ta, trans_b=tb, m_live=cnt)
    full = ops.gemm_x6(a, b, trans_a=ta, trans_b=tb)
    assert torch.equal(outs["on"], outs["off"])
    assert torch.equal(outs["on"], full)
    ref, mag = _ref(a, b, ta, tb)
    err = (outs["on"].double() - ref).abs()
    assert (err <= 2e-6 * mag + 1e-30).all(), float((err / (mag + 1e-30)).max())


@pytest.mark.parametrize("H,dropout", [(512, 0.5), (128, 0.0)])
def test_wide_ln_act_live_rows_bitwise(H, dropout):
    """ops.wide_ln_act with a live-row count (layer 0 of the wide NS model): the live rows'
    outputs and input gradients, and the bias / LayerNorm gradients, bitwise those of the
    all-rows launch when the incoming gradient is zero past the live rows (the skipped rows only
    added exact zeros to the partials)."""
    from regnn_hip import ops
    g = torch.Generator(device=DEV).manual_seed(H)
    n, live = 13312, 4900
    x0 = torch.randn(n, H, generator=g, device=DEV)
    x0[live:] = 0
    rs = torch.rand(n, generator=g, device=DEV) + 0.5
    gy = torch.randn(n, H, generator=g, device=DEV)
    gy[live:] = 0
    state = torch.tensor([3, 5, 7, 9, 11, 0, 0, 0], dtype=torch.int64, device=DEV)
    cnt = torch.tensor([live], dtype=torch.int32, device=DEV)
    outs = []
    for lv in (None, cnt):
        ln = torch.nn.LayerNorm(H).to(DEV)
        with torch.no_grad():
            ln.weight.copy_(torch.linspace(0.5, 1.5, H, device=DEV))
            ln.bias.copy_(torch.linspace(-0.2, 0.2, H, device=DEV))
        bias = torch.linspace(-0.1, 0.1, H, device=DEV).requires_grad_(True)
        x = x0.clone().requires_grad_(True)
        y = ops.wide_ln_act(x, bias, ln, p=dropout, state=state, layer=0, rs=rs, live=lv)
        y.backward(gy)
        outs.append((y[:live].detach().clone(), x.grad.clone(), bias.grad.clone(),
                     ln.weight.grad.clone(), ln.bias.grad.clone()))
    for name, a, b in zip(["y", "gx", "g_bias", "g_gamma", "g_beta"], outs[0], outs[1]):
        assert torch.equal(a, b), name
    assert not outs[1][1][live:].any()             # the dead rows' gradient: zeros
