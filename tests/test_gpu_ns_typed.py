"""Layer 0 of the NS REGNN with group_input folded in (mag.REGNN._typed_first_layer over
regnn_ns_typed_agg): the raw input rows aggregated per source node type, projected after the mean
by the composed W_t^T W_0 -- the module path at any hidden width (the reference default hidden
512, mag/regnn_ns.py:43). Loss and every parameter gradient must equal the reference-ordered path
(group_input over every sampled node, then x_src @ W, then the mean: mag/regnn_ns.py:300-346,
mag/regnn_layers.py:101-148) on the same sampled batch."""
import os
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import _golden as G  # noqa: E402
from test_gpu_ns_engine import _mag, DEV  # noqa: E402


def _grads_one_step(d, hidden, typed, dropout, residual=False, batch=96, sizes=(6, 4),
                    pre=None, strided=None):
    from regnn_hip import mag, ns, ops
    from regnn_hip.ns import NSTrainer
    old, old_csc = mag.TYPED_AGG["mode"], ops.NS_CSC["mode"]
    old_pre, old_str = ns.MODULE_PRE_SUMS["mode"], ns.MODULE_STRIDED["mode"]
    if pre is not None:
        ns.MODULE_PRE_SUMS["mode"] = "on" if pre else "off"
    if strided is not None:
        ns.MODULE_STRIDED["mode"] = "on" if strided else "off"
    # the reference-ordered run also takes the atomic scatter backward of the last layer
    mag.TYPED_AGG["mode"] = ops.NS_CSC["mode"] = "auto" if typed else "off"
    try:
        torch.manual_seed(7)
        K = int(d["x_dict"][0].shape[1])
        m = mag.REGNN(K, hidden, 13, 2, 10.0, dropout, {k: K for k in d["x_dict"]}, 7,
                      use_norm="ln", self_loop_type=2, residual=residual).to(DEV)
        with torch.no_grad():
            for conv in m.convs:
                conv.relation_weight.copy_(torch.linspace(-0.02, 0.12, conv.relation_weight.numel(),
                                                            device=DEV))
                conv.bias.normal_(0, 0.1)
        m.train()
        opt = torch.optim.SGD(m.parameters(), lr=0.0)
        tr = NSTrainer(m, opt, d["rg"], list(sizes), batch, torch.arange(d["n_paper"], device=DEV),
                       d["x_dict"], d["edge_type"], d["node_type"], d["local"], d["y"], 7, seed=3,
                       engine="module")
        seen = []
        orig = m._typed_first_layer

        def spy(*a, **k):
            out = orig(*a, **k)
            seen.append(out is not None)
            return out
        m._typed_first_layer = spy
        torch.manual_seed(11)                  # the model-level dropout's torch RNG
        tr._forward_backward()
        torch.cuda.synchronize()
        assert seen == [typed]
        if strided is not None:                # hop 0's layout
            assert all((getattr(s.blocks[0], "strided_rows", None) is not None) == strided
                       for s in tr.slots)
        if pre is not None:                    # the outer hop's sums path ran (or not)
            assert all((s.typed_sums[-1] is not None) == pre for s in tr.slots)
            assert all(s.sums_fresh[-1] == pre for s in tr.slots[:1])
        return float(tr.loss), {n: p.grad.detach().double().cpu().numpy().copy()
                                for n, p in m.named_parameters()}
    finally:
        mag.TYPED_AGG["mode"], ops.NS_CSC["mode"] = old, old_csc
        ns.MODULE_PRE_SUMS["mode"], ns.MODULE_STRIDED["mode"] = old_pre, old_str


@pytest.mark.parametrize("K,hidden,residual", [(128, 512, False), (128, 64, False),
                                               (64, 128, True), (128, 256, False)])
def test_typed_first_layer_matches_reference_order(K, hidden, residual):
    d = _mag(0.003, seed=2, F=K)
    la, ga = _grads_one_step(d, hidden, True, 0.0, residual)
    lb, gb = _grads_one_step(d, hidden, False, 0.0, residual)
    assert abs(la - lb) <= 1e-5 * max(1.0, abs(lb)), (la, lb)
    for n in gb:
        ok, err = G.close(ga[n], gb[n], 1e-5)
        assert ok, f"{n}: rel err {err:.3e}"
    # the relation table of layer 0 has a gradient through the typed aggregation
    assert np.abs(ga["convs.0.relation_weight"]).max() > 0


@pytest.mark.parametrize("hidden,dropout", [(512, 0.0), (64, 0.0), (256, 0.5)])
def test_module_pre_sums_match_typed_agg(hidden, dropout):
    """the module path's layer 0 from the sampler's per-type input sums (relation slots: the outer
    hop as regnn_ns_hop_typed_sums, ops.ns_slot_agg) against the same layer gathering the sampled
    raw rows itself (regnn_ns_typed_agg): the same batch, loss and every gradient at 1e-5."""
    d = _mag(0.003, seed=4, F=128)
    la, ga = _grads_one_step(d, hidden, True, dropout, pre=True)
    lb, gb = _grads_one_step(d, hidden, True, dropout, pre=False)
    assert abs(la - lb) <= 1e-5 * max(1.0, abs(lb)), (la, lb)
    for n in gb:
        ok, err = G.close(ga[n], gb[n], 1e-5)
        assert ok, f"{n}: rel err {err:.3e}"
    assert np.abs(ga["convs.0.relation_weight"]).max() > 0


@pytest.mark.parametrize("hidden,typed", [(512, True), (64, True), (128, True)])
def test_module_strided_hop0_matches_csr(hidden, typed):
    """the module path's hop 0 in the strided layout (the last layer's forward over rows at i S,
    regnn_ns_spmm_strided_fwd; its backward over the transposed index the strided hop builds)
    against hop 0 in the CSR layout: the same batch, loss and every gradient at 1e-5."""
    d = _mag(0.003, seed=5, F=128)
    la, ga = _grads_one_step(d, hidden, typed, 0.0, strided=True)
    lb, gb = _grads_one_step(d, hidden, typed, 0.0, strided=False)
    assert abs(la - lb) <= 1e-5 * max(1.0, abs(lb)), (la, lb)
    for n in gb:
        ok, err = G.close(ga[n], gb[n], 1e-5)
        assert ok, f"{n}: rel err {err:.3e}"


def _three_types(d):
    """the same graph with 3 node types (institution and field merged into one type, their
    feature tables concatenated): T = 3 is not a multiple of 4, so [S | w] rows carry pad
    columns (ops.ns_typed_agg ext)."""
    nt = d["node_type"].clone()
    n2 = int(d["x_dict"][2].shape[0])
    local = d["local"].clone()
    f = nt == 3
    local[f] += n2
    nt[f] = 2
    x = {0: d["x_dict"][0], 1: d["x_dict"][1],
         2: torch.cat([d["x_dict"][2], d["x_dict"][3]], 0).contiguous()}
    return dict(d, node_type=nt, local=local, x_dict=x)


@pytest.mark.parametrize("hidden", [64, 512])
def test_typed_first_layer_three_types(hidden):
    """T = 3 node types (row stride T K + 4, not T K + T) through the typed first
    layer, against the reference-ordered path."""
    d = _three_types(_mag(0.003, seed=2, F=128))
    la, ga = _grads_one_step(d, hidden, True, 0.0)
    lb, gb = _grads_one_step(d, hidden, False, 0.0)
    assert abs(la - lb) <= 1e-5 * max(1.0, abs(lb)), (la, lb)
    for n in gb:
        ok, err = G.close(ga[n], gb[n], 1e-5)
        assert ok, f"{n}: rel err {err:.3e}"
    assert np.abs(ga["convs.0.relation_weight"]).max() > 0


def test_typed_agg_against_fp64_sums():
    """S / w rows of regnn_ns_typed_agg against fp64 sums over the block's CSR rows, and its
    relation-table gradient against autograd of the fp64 restatement."""
    from regnn_hip import ops
    from regnn_hip.ns import DeviceSampler
    d = _mag(0.003, seed=4, F=128)
    s = DeviceSampler(d["rg"], [6, 4], 64, etype=d["edge_type"], ntype=d["node_type"],
                      num_edge_types=7)
    s.set_seed(5, 0, 1)
    s.set_targets(torch.arange(64, device=DEV) * 3)
    s.run_hops(meta_only=False, strided=False)
    blk = s.blocks[1]                           # layer 0's block (the outer hop)
    sz = s.sizes.cpu().tolist()
    n_dst, E = sz[1], sz[9]
    tables = [d["x_dict"][k] for k in range(4)]
    rw = torch.linspace(-0.05, 0.2, 11, device=DEV, requires_grad=True)
    tab = torch.nn.functional.leaky_relu(rw * 10.0)
    n_id = s.n_id.to(torch.int64)
    S, w = ops.ns_typed_agg(blk, tab, n_id, tables, d["node_type"], d["local"])
    gS = torch.randn_like(S)
    gw = torch.randn_like(w)
    (S * gS).sum().add((w * gw).sum()).backward()
    # fp64 restatement
    ptr = blk.csr_ptr[:n_dst + 1].cpu().numpy()
    idx = blk.csr_idx[:E].cpu().numpy()
    rel = blk.rel[:E].cpu().numpy().astype(np.int64)
    nid = n_id.cpu().numpy()
    nt = d["node_type"].cpu().numpy()
    lo = d["local"].cpu().numpy()
    X = [t.double().cpu().numpy() for t in tables]
    rw64 = torch.tensor(rw.detach().cpu().numpy(), dtype=torch.float64, requires_grad=True)
    tab64 = torch.nn.functional.leaky_relu(rw64 * 10.0)
    e_dst = np.repeat(np.arange(n_dst), np.diff(ptr))
    g_src = nid[idx]
    e_t = nt[g_src]
    e_x = np.stack([X[e_t[i]][lo[g_src[i]]] for i in range(E)])
    wt = tab64[torch.from_numpy(rel)]
    S64 = torch.zeros(n_dst, 4, 128, dtype=torch.float64)
    w64 = torch.zeros(n_dst, 4, dtype=torch.float64)
    flat = torch.from_numpy(e_dst * 4 + e_t)
    S64.view(-1, 128).index_add_(0, flat, wt[:, None] * torch.from_numpy(e_x))
    w64.view(-1).index_add_(0, flat, wt)
    ok, err = G.close(S[:n_dst].detach().cpu().numpy(), S64.detach().numpy(), 1e-5)
    assert ok, err
    ok, err = G.close(w[:n_dst].detach().cpu().numpy(), w64.detach().numpy(), 1e-5)
    assert ok, err
    ((S64 * gS[:n_dst].double().cpu()).sum() + (w64 * gw[:n_dst].double().cpu()).sum()).backward()
    ok, err = G.close(rw.grad.cpu().numpy(), rw64.grad.numpy(), 1e-5)
    assert ok, err
    # the [S | w] form (one strided operand): the same values, the same relation-table gradient
    g_ref = rw.grad.clone()
    rw.grad = None
    tab = torch.nn.functional.leaky_relu(rw * 10.0)
    Sw = ops.ns_typed_agg(blk, tab, n_id, tables, d["node_type"], d["local"], ext=True)
    assert Sw.shape == (S.shape[0], 4 * 128 + 4)
    assert torch.equal(Sw[:, :512], S.detach().reshape(S.shape[0], 512))
    assert torch.equal(Sw[:, 512:], w.detach())
    (Sw * torch.cat([gS.reshape(gS.shape[0], 512), gw], 1)).sum().backward()
    assert torch.equal(rw.grad, g_ref)


@pytest.mark.parametrize("dropout", [0.0, 0.5])
@pytest.mark.parametrize("hidden,residual", [(256, False), (512, True)])
def test_wide_epilogue_and_gemm_match_torch_path(monkeypatch, hidden, residual, dropout):
    """the wide module path's one-launch epilogue (ops.wide_ln_act: bias /
    residual / LayerNorm / relu / dropout forward and backward) and its fp32-accurate bf16x6
    GEMMs (ops.mm) against the same step on torch's kernels (hipBLASLt fp32, LayerNorm, relu,
    dropout), loss and every gradient at 1e-5. With dropout the torch run gets the epilogue's
    hash masks (oracle.dropout_mask of the fused step's per-layer key) in place of torch's RNG."""
    from oracle import regnn_oracle as O
    from regnn_hip import mag, ops
    from test_gpu_ns_engine import _nsm_seed
    d = _mag(0.003, seed=4, F=128)

    def run(fast):
        monkeypatch.setitem(mag.WIDE_EPI, "mode", "on" if fast else "off")
        monkeypatch.setitem(ops.GEMM_X6, "mode", "on" if fast else "off")
        calls = []
        if not fast and dropout > 0:
            keep16 = int(round((1 - dropout) * 65536))
            real = torch.nn.functional.dropout

            def hash_dropout(x, p=0.5, training=True, inplace=False):
                if not training or p == 0:
                    return real(x, p, training, inplace)
                layer = len(calls)
                calls.append(layer)
                st = tr_box[0].sampler.state.cpu().tolist()
                mask = O.dropout_mask(_nsm_seed(st, layer), x.shape[0], x.shape[1], 4, keep16)
                return x * torch.from_numpy(mask).to(x.device, x.dtype) / (keep16 / 65536)
            monkeypatch.setattr(torch.nn.functional, "dropout", hash_dropout)
        from regnn_hip.ns import NSTrainer
        torch.manual_seed(7)
        m = mag.REGNN(128, hidden, 13, 2, 10.0, dropout, {k: 128 for k in d["x_dict"]}, 7,
                      use_norm="ln", self_loop_type=2, residual=residual).to(DEV)
        with torch.no_grad():
            for conv in m.convs:
                conv.relation_weight.copy_(torch.linspace(-0.02, 0.12, conv.relation_weight.numel(),
                                                            device=DEV))
                conv.bias.normal_(0, 0.1)
                conv.norm.weight.normal_(1, 0.1)
        m.train()
        tr = NSTrainer(m, None, d["rg"], [6, 4], 96, torch.arange(d["n_paper"], device=DEV),
                       d["x_dict"], d["edge_type"], d["node_type"], d["local"], d["y"], 7, seed=3,
                       engine="module", pipeline=False)
        tr_box[0] = tr
        tr._forward_backward()
        torch.cuda.synchronize()
        if not fast and dropout > 0:
            assert calls == [0, 1]
        monkeypatch.undo()
        return float(tr.loss), {n: p.grad.detach().double().cpu().numpy().copy()
                                for n, p in m.named_parameters()}

    tr_box = [None]
    la, ga = run(True)
    lb, gb = run(False)
    assert abs(la - lb) <= 1e-5 * max(1.0, abs(lb)), (la, lb)
    for n in gb:
        ok, err = G.close(ga[n], gb[n], 1e-5)
        assert ok, f"{n}: rel err {err:.3e}"


def test_csc_gather_chunked_hubs_match(monkeypatch):
    """the module path's transposed gather with the hub rows chunked over the grid
    (regnn_ns_spmm_bwd_csc hub_work, NS_CSC_CHUNKED on) against a workgroup per hub row: loss and
    every gradient at 1e-5 (fan-out 25 makes hubs of hundreds of entries at batch 512)."""
    from regnn_hip import ops
    d = _mag(0.01, seed=5, F=128)
    out = {}
    for mode in ("on", "off"):
        monkeypatch.setitem(ops.NS_CSC_CHUNKED, "mode", mode)
        out[mode] = _grads_one_step(d, 256, True, 0.0, batch=512, sizes=(25, 20))
    la, ga = out["on"]
    lb, gb = out["off"]
    assert abs(la - lb) <= 1e-5 * max(1.0, abs(lb))
    for n in gb:
        ok, err = G.close(ga[n], gb[n], 1e-5)
        assert ok, f"{n}: rel err {err:.3e}"



def test_rel_tab_and_labels_match_torch():
    """the module path's one-launch helpers against the torch ops they replace: the relation
    table leaky_relu(alpha rw) (mag/regnn_layers.py:110-111, forward bitwise, backward to 1e-6)
    and the batch's labels with -100 past the live targets (mag/regnn_ns.py:404)."""
    import torch.nn.functional as F
    from regnn_hip import ops
    g0 = torch.Generator(device=DEV)
    g0.manual_seed(7)
    rw = (torch.randn(23, device=DEV, generator=g0) * 0.02).requires_grad_(True)
    ref_rw = rw.detach().clone().requires_grad_(True)
    tab = ops.rel_tab(rw, 100.0)
    ref = F.leaky_relu(ref_rw * 100.0)
    assert torch.equal(tab, ref)
    g = torch.randn(23, device=DEV, generator=g0)
    tab.backward(g)
    ref.backward(g)
    torch.testing.assert_close(rw.grad, ref_rw.grad, rtol=1e-6, atol=0)
    n_id = torch.randint(0, 1000, (64,), device=DEV, dtype=torch.int32, generator=g0)
    labels = torch.randint(0, 349, (1000,), device=DEV, generator=g0)
    for live in (0, 50, 64):
        sizes = torch.tensor([live], device=DEV, dtype=torch.int32)
        y = ops.ns_labels(n_id, sizes, labels, 64)
        want = torch.where(torch.arange(64, device=DEV) < live, labels[n_id.long()],
                           torch.full((64,), -100, device=DEV))
        assert torch.equal(y, want)


def test_rel_tabs_match_torch():
    """ops.rel_tabs: every layer's relation table from one launch, forward bitwise against
    leaky_relu(alpha rw) per table (mag/regnn_layers.py:110-111), backward per table to 1e-6,
    a table the loss does not reach getting a zero gradient."""
    import torch.nn.functional as F
    from regnn_hip import ops
    g0 = torch.Generator(device=DEV)
    g0.manual_seed(11)
    for sizes in ((23,), (23, 23, 23), (5, 300, 1, 17)):
        rws = [(torch.randn(n, device=DEV, generator=g0) * 0.02).requires_grad_(True)
               for n in sizes]
        refs = [r.detach().clone().requires_grad_(True) for r in rws]
        tabs = ops.rel_tabs(rws, 100.0)
        want = [F.leaky_relu(r * 100.0) for r in refs]
        for t, w in zip(tabs, want):
            assert torch.equal(t, w)
        gs = [torch.randn(n, device=DEV, generator=g0) for n in sizes]
        used = range(len(sizes) - 1) if len(sizes) > 1 else range(1)
        sum((tabs[i] * gs[i]).sum() for i in used).backward()
        sum((want[i] * gs[i]).sum() for i in used).backward()
        for i, (r, rr) in enumerate(zip(rws, refs)):
            if i in used:
                torch.testing.assert_close(r.grad, rr.grad, rtol=1e-6, atol=0)
            else:
                assert r.grad is None or not r.grad.any()


def test_softmax_xent_matches_torch():
    """ops.softmax_xent (one launch each way) against log_softmax + nll_loss with ignored rows,
    loss and logits gradient to 1e-6, and the all-ignored batch (nan, as torch)."""
    import torch.nn.functional as F
    from regnn_hip import ops
    g0 = torch.Generator(device=DEV)
    g0.manual_seed(3)
    for B, C in ((512, 349), (37, 5), (1, 64)):
        z = (torch.randn(B, C, device=DEV, generator=g0) * 3).requires_grad_(True)
        y = torch.randint(0, C, (B,), device=DEV, generator=g0)
        y[::7] = -100
        if B == 1:
            y[0] = 3
        zr = z.detach().clone().requires_grad_(True)
        loss = ops.softmax_xent(z, y)
        ref = F.nll_loss(zr.log_softmax(-1), y)
        torch.testing.assert_close(loss, ref, rtol=1e-6, atol=1e-6)
        loss.backward()
        ref.backward()
        torch.testing.assert_close(z.grad, zr.grad, rtol=1e-5, atol=1e-7)
    z = torch.randn(4, 6, device=DEV)
    assert torch.isnan(ops.softmax_xent(z, torch.full((4,), -100, device=DEV)))


@pytest.mark.parametrize("B,K,C,live", [(512, 512, 349, 300), (512, 64, 349, 512), (37, 128, 5, 0),
                                        (1, 64, 64, 1), (1030, 64, 17, 1000)])
def test_ns_lin_xent_matches_torch(B, K, C, live):
    """ops.ns_lin_xent (out_lin GEMM, then labels + per-row loss + the fixed-order mean in one
    launch; backward: gz and out_lin's bias gradient in one launch) against F.linear +
    log_softmax + nll_loss over labels[n_id[:B]] with the rows past sizes[0] ignored (and the
    labelled -100 rows): loss, x / W / b gradients to 1e-5; the ticket is back at zero after each
    call (repeat calls agree bitwise); live 0: every row ignored -> nan, as torch."""
    import torch.nn.functional as F
    from regnn_hip import ops
    g0 = torch.Generator(device=DEV)
    g0.manual_seed(11)
    n_lab = 5000
    labels = torch.randint(0, C, (n_lab,), device=DEV, generator=g0)
    labels[::13] = -100
    n_id = torch.randint(0, n_lab, (B,), device=DEV, generator=g0).to(torch.int32)
    sizes = torch.tensor([live, 0, 0, 0], dtype=torch.int32, device=DEV)
    x = torch.randn(B, K, device=DEV, generator=g0).requires_grad_(True)
    lin = torch.nn.Linear(K, C).to(DEV)
    ticket = torch.zeros(1, dtype=torch.int32, device=DEV)
    y = labels[n_id.long()].clone()
    y[live:] = -100
    xr = x.detach().clone().requires_grad_(True)
    wr = lin.weight.detach().clone().requires_grad_(True)
    br = lin.bias.detach().clone().requires_grad_(True)
    ref = F.nll_loss(F.linear(xr, wr, br).log_softmax(-1), y)
    loss = ops.ns_lin_xent(x, lin.weight, lin.bias, n_id, sizes, labels, ticket)
    if live == 0 or bool((y == -100).all()):
        assert torch.isnan(loss) and torch.isnan(ref)
        return
    torch.testing.assert_close(loss, ref, rtol=1e-5, atol=1e-6)
    loss.backward()
    ref.backward()
    torch.testing.assert_close(x.grad, xr.grad, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(lin.weight.grad, wr.grad, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(lin.bias.grad, br.grad, rtol=1e-5, atol=1e-6)
    torch.cuda.synchronize()
    assert int(ticket.item()) == 0
    again = ops.ns_lin_xent(x, lin.weight, lin.bias, n_id, sizes, labels, ticket)
    assert float(again) == float(loss) and int(ticket.item()) == 0
