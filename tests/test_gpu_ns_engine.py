"""GPU checks of the device-resident NS step (regnn_hip.ns: regnn_ns_batch / regnn_ns_hop /
regnn_ns_spmm_bwd, mag/regnn_ns.py:206-214,392-420):

* the capacity-sized sampler is bit-exact against oracle/sampler_oracle.py (n_id, edge lists,
  e_id, block layout) including a partial last batch;
* one NSTrainer step (no host sizes) gives the same loss and parameter gradients as the
  PyG-style path (NeighborSampler + mag.train_step) on the same batch;
* the HIP-graph replay of the step tracks the eager step;
* data parallelism: the gradient of the union batch equals the mean of its two halves'
  gradients (the DP all-reduce's contract);
* one step at the BASELINE config-5 scale (mag_like(10), batch 512, fan-out [25, 20]): sampled
  rows against the oracle spec, sampler properties, and block aggregation rows against fp64.
"""
import numpy as np
import pytest
import torch

import _golden as G
from oracle import sampler_oracle as SO

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _mag(scale, seed=0, F=16, hidden=32, classes=5, dropout=0.0):
    from regnn_hip import mag, synth
    from regnn_hip.graph import RelGraph
    gd = synth.mag_like(scale, seed=seed, device=DEV)
    keep = gd["rel"] <= 7
    rg = RelGraph(gd["src"][keep], gd["dst"][keep], gd["N"], DEV)
    edge_type = gd["rel"][keep].to(torch.int64) - 1
    del keep
    node_type = gd["ntype"]
    offs = torch.tensor([gd["type_offsets"][t] for t in synth.NTYPES], device=DEV)
    local = torch.arange(gd["N"], device=DEV) - offs[node_type]
    feats = synth.type_features(gd["counts"], {t: F for t in synth.NTYPES}, seed=1, device=DEV)
    x_dict = {k: f for k, f in enumerate(feats)}
    n_paper = gd["counts"]["paper"]
    y = torch.full((gd["N"], 1), -1, dtype=torch.int64, device=DEV)
    y[:n_paper, 0] = (torch.arange(n_paper, device=DEV) * 7) % classes

    def model(seed=0):
        torch.manual_seed(seed)
        m = mag.REGNN(F, hidden, classes, 2, 10.0, dropout, {k: F for k in x_dict}, 7,
                      use_norm="ln", self_loop_type=2).to(DEV)
        with torch.no_grad():
            for conv in m.convs:
                conv.relation_weight.copy_(torch.linspace(0.02, 0.12, 11, device=DEV))
                conv.bias.normal_(0, 0.1)
        return m

    return dict(gd=gd, rg=rg, edge_type=edge_type, node_type=node_type, local=local,
                x_dict=x_dict, y=y, n_paper=n_paper, model=model)


def _oracle_csr(rg):
    return rg.csr_ptr.cpu().numpy(), rg.csr_idx.cpu().numpy(), rg.csr_eid.cpu().numpy()


def test_device_sampler_bit_exact_partial_batch():
    from regnn_hip.graph import RelGraph
    from regnn_hip.ns import DeviceSampler
    rng = np.random.default_rng(3)
    N, E = 4000, 60000
    dst = np.minimum((rng.pareto(1.1, E) * 4).astype(np.int64), N - 1)
    src = rng.integers(0, N, E)
    et = rng.integers(0, 7, E)
    nt = rng.integers(0, 4, N)
    rg = RelGraph(src, dst, N, DEV)
    ptr, idx, eid = _oracle_csr(rg)
    ds = DeviceSampler(rg, [9, 5], 100, etype=torch.from_numpy(et), ntype=torch.from_numpy(nt),
                       num_edge_types=7)
    for bi, batch in enumerate([np.arange(0, 100), rng.permutation(N)[:37], np.array([11])]):
        ds.set_seed(99, 2, bi)
        ds.set_targets(torch.from_numpy(batch).to(DEV))
        ds.run_hops()
        n_total, hops = ds.exact_adjs()
        _, rn_id, radjs = SO.neighbor_sample(ptr, idx, batch.tolist(), [9, 5], 99, epoch=2,
                                             batch_idx=bi)
        assert ds.n_id[:n_total].cpu().tolist() == rn_id
        for (ei, e_id, size, blk, cnt), (s, d, e, rsize) in zip(hops, radjs[::-1]):
            assert tuple(size) == tuple(rsize)
            assert ei[0].cpu().tolist() == s and ei[1].cpu().tolist() == d
            assert e_id.cpu().tolist() == [int(eid[p]) for p in e]
            # block layout: row v = its sampled edges in order, then its self loop
            p_ = blk.csr_ptr.cpu().numpy()
            ix, rl, ps = blk.csr_idx.cpu().numpy(), blk.rel.cpu().numpy(), blk.pos.cpu().numpy()
            n_dst = size[1]
            tgt = np.asarray(rn_id[:n_dst])
            assert p_[0] == 0 and np.all(np.diff(p_) == cnt.cpu().numpy() + 1)
            assert np.all(ix[p_[1:] - 1] == np.arange(n_dst))
            assert np.all(rl[p_[1:] - 1] == 7 + nt[tgt])
            keep = ps >= 0
            assert np.all(rl[keep] == et[eid[ps[keep]]])
            inv = blk.inv.cpu().numpy()
            assert np.allclose(inv, 1.0 / np.diff(p_))


def _setup_trainer(d, model, batch=64, sizes=(6, 4), seed=3, lr=1e-2):
    from regnn_hip.ns import NSTrainer
    opt = torch.optim.Adam(model.parameters(), lr=lr, capturable=True)
    return NSTrainer(model, opt, d["rg"], list(sizes), batch,
                     torch.arange(d["n_paper"], device=DEV), d["x_dict"], d["edge_type"],
                     d["node_type"], d["local"], d["y"], 7, seed=seed), opt


def test_trainer_step_matches_pyg_path():
    """one device-engine step == NeighborSampler + mag.train_step on the same batch (loss and
    every parameter gradient at 1e-5)."""
    from regnn_hip import mag
    from regnn_hip.sampler import NeighborSampler
    d = _mag(0.003, seed=1)
    m_api, m_eng = d["model"](), d["model"]()
    m_api.train(); m_eng.train()
    smp = NeighborSampler(d["rg"], torch.arange(d["n_paper"], device=DEV), [6, 4], batch_size=64,
                          shuffle=True, seed=3)
    batch = next(iter(smp))
    opt_api = torch.optim.SGD(m_api.parameters(), lr=0.0)
    loss_api = mag.train_step(m_api, opt_api, batch, d["x_dict"], d["edge_type"], d["node_type"],
                              d["local"], d["y"], 1)
    tr, _ = _setup_trainer(d, m_eng)
    tr._forward_backward()
    torch.cuda.synchronize()
    assert abs(float(tr.loss) - float(loss_api.detach())) <= 1e-5 * max(1.0, abs(float(loss_api.detach())))
    assert int(tr.sampler.sizes[0]) == 64
    gp = dict(m_api.named_parameters())
    for n, p in m_eng.named_parameters():
        if gp[n].grad is None:                 # declared, unused in forward (REGNN.norm)
            assert not p.grad.any(), n
            continue
        ok, err = G.close(p.grad.cpu().numpy(), gp[n].grad.cpu().numpy().astype(np.float64), 1e-5)
        assert ok, f"{n}: rel err {err:.3e}"


@pytest.mark.parametrize("model_kind", ["regat", "regcn_sl1"])
def test_trainer_module_path_other_models(model_kind):
    """NSTrainer's module path for the REGNN convs the device blocks do not cover (mag REGATConv;
    REGCNConv with self_loop_type 1): exact-size PyG adjs and the real edge types, the same loss
    and gradients as NeighborSampler + mag.train_step on the same batch; capture() refuses."""
    from regnn_hip import mag
    from regnn_hip.sampler import NeighborSampler
    d = _mag(0.003, seed=1)

    def make():
        torch.manual_seed(0)
        if model_kind == "regat":
            return mag.REGNN(16, 8, 5, 2, 10.0, 0.0, {k: 16 for k in d["x_dict"]}, 7,
                             use_norm="ln", self_loop_type=2, model="regat", heads=2).to(DEV)
        return mag.REGNN(16, 32, 5, 2, 10.0, 0.0, {k: 16 for k in d["x_dict"]}, 7,
                         use_norm="ln", self_loop_type=1).to(DEV)
    m_api, m_eng = make(), make()
    smp = NeighborSampler(d["rg"], torch.arange(d["n_paper"], device=DEV), [6, 4], batch_size=64,
                          shuffle=True, seed=3)
    batch = next(iter(smp))
    loss_api = mag.train_step(m_api, torch.optim.SGD(m_api.parameters(), lr=0.0), batch,
                              d["x_dict"], d["edge_type"], d["node_type"], d["local"], d["y"], 1)
    tr, _ = _setup_trainer(d, m_eng)
    assert tr.fused is None
    tr._forward_backward()
    torch.cuda.synchronize()
    la = float(loss_api.detach())
    assert abs(float(tr.loss) - la) <= 1e-5 * max(1.0, abs(la))
    gp = dict(m_api.named_parameters())
    for n, p in m_eng.named_parameters():
        if gp[n].grad is None:
            assert not p.grad.any(), n
            continue
        ok, err = G.close(p.grad.cpu().numpy(), gp[n].grad.cpu().numpy().astype(np.float64), 1e-5)
        assert ok, f"{n}: rel err {err:.3e}"
    with pytest.raises(ValueError):
        tr.capture(warmup=1)


def test_trainer_graph_replay_tracks_eager():
    d = _mag(0.003, seed=2)
    tr_e, _ = _setup_trainer(d, d["model"](7), batch=128, sizes=(10, 5))
    tr_g, _ = _setup_trainer(d, d["model"](7), batch=128, sizes=(10, 5))
    # capture() undoes its warm-up steps: the first replay trains the epoch's first batch
    tr_g.capture(warmup=2)
    le, lg = [], []
    for _ in range(6):
        tr_e.step()
        le.append(float(tr_e.loss))
        tr_g.replay()
        lg.append(float(tr_g.loss))
    assert np.all(np.isfinite(lg))
    assert np.allclose(le, lg, rtol=1e-4, atol=1e-5), (le, lg)
    assert tr_g.edges_total() > 0


@pytest.mark.parametrize("graph,engine", [(False, "fused"), (True, "fused"), (False, "module"),
                                          (True, "module"), (True, "module1")])
def test_pipelined_trainer_matches_unpipelined(monkeypatch, graph, engine):
    """sampler slots filled ahead on a second stream while the model trains give the
    unpipelined batch sequence, dropout masks and losses, across an epoch change; for the fused
    step and for the module path at hidden 128 (the typed first layer, meta-only last hop;
    dropout off: the module path draws torch's RNG) at its default lookahead and at 1
    ("module1": the next batch only)."""
    from regnn_hip import ns
    from regnn_hip.ns import NSTrainer
    monkeypatch.setitem(ns.MODULE_PIPELINE, "mode", "on")
    if engine == "module1":
        monkeypatch.setitem(ns.MODULE_AHEAD, "n", 1)
    fused = engine == "fused"
    d = _mag(0.002, seed=8, F=128, hidden=64 if fused else 128, classes=13,
             dropout=0.4 if fused else 0.0)

    def make(pipe):
        return NSTrainer(d["model"](5), None, d["rg"], [6, 4], 100,
                         torch.arange(d["n_paper"], device=DEV), d["x_dict"], d["edge_type"],
                         d["node_type"], d["local"], d["y"], 7, seed=9, adam=dict(lr=1e-2),
                         pipeline=pipe)
    tr_p, tr_u = make(True), make(False)
    assert tr_p.pipelined and not tr_u.pipelined
    assert (tr_p.fused is not None) == fused and (fused or tr_p._module_lean)
    if graph:
        tr_p.capture(warmup=2)                          # warm-up steps undone by capture()
    run_p = tr_p.replay if graph else tr_p.step
    lp, lu = [], []
    for i in range(7):
        if i == 4:                                      # an epoch change mid-run
            tr_p.set_epoch(1)
            tr_u.set_epoch(1)
        run_p()
        tr_u.step()
        assert torch.equal(tr_p.sampler.n_id[:int(tr_p.sampler.sizes[0])],
                           tr_u.sampler.n_id[:int(tr_u.sampler.sizes[0])])
        lp.append(float(tr_p.loss))
        lu.append(float(tr_u.loss))
    assert np.all(np.isfinite(lp))
    # the module path's small products run on hipBLASLt, which may pick another algorithm when
    # captured than eagerly (ulp-level differences that Adam carries forward): 1e-5 there
    tol = 1e-6 if fused else 5e-5
    assert np.allclose(lp, lu, rtol=tol, atol=tol * 0.1), (lp, lu)


def test_module_run_steps_groups_match_single_replays(monkeypatch):
    """the module path's lookahead groups (MODULE_AHEAD 4: 8 slots, 4- and 2-step graphs whose
    sampler fills the other slots, one fork and one join per group) train the same batches to
    the same losses and parameters as one-step replays, across an epoch boundary."""
    d = _mag(0.002, seed=8, F=128, hidden=128, classes=13, dropout=0.0)
    from regnn_hip import ns
    from regnn_hip.ns import NSTrainer
    monkeypatch.setitem(ns.MODULE_PIPELINE, "mode", "on")
    monkeypatch.setitem(ns.MODULE_AHEAD, "n", 4)

    def make():
        return NSTrainer(d["model"](5), None, d["rg"], [6, 4], 100,
                         torch.arange(d["n_paper"], device=DEV), d["x_dict"], d["edge_type"],
                         d["node_type"], d["local"], d["y"], 7, seed=9, adam=dict(lr=1e-2),
                         engine="module")
    ta, tb = make(), make()
    assert ta.fused is None and ta._module_lean
    ta.capture(warmup=1)
    tb.capture(warmup=1)
    assert ta.ahead == 4 and len(ta.slots) == 8
    assert sorted(ta.graph_groups) == [(m, c) for m in (2, 4) for c in range(8)]
    # (hipBLASLt's small products may differ by ulps between graphs, and Adam's m / sqrt(v)
    # turns an ulp in a near-zero gradient into up to a fraction of its step lr = 1e-2: a few
    # parameters differ by ~5e-5 after 4 steps, the losses stay bitwise equal; 1e-3 = lr / 10)
    for k in (4, 3, 2, 7):
        ta.run_steps(k)
        for _ in range(k):
            tb.replay()
        torch.cuda.synchronize()
        assert ta.cur == tb.cur and ta._trained == tb._trained
        assert torch.equal(ta.sampler.n_id[:int(ta.sampler.sizes[0])],
                           tb.sampler.n_id[:int(tb.sampler.sizes[0])])
        assert abs(float(ta.loss) - float(tb.loss)) <= 5e-5 * abs(float(tb.loss))
        dd = (ta.pflat - tb.pflat).abs()
        assert float(dd.max()) <= 1e-3, \
            (k, float(dd.max()), int((dd > 1e-6).sum()), ta.pflat.numel(), float(ta.loss),
             float(tb.loss))
    ta.set_epoch(1)
    tb.set_epoch(1)
    ta.run_steps(2)
    tb.replay(); tb.replay()
    torch.cuda.synchronize()
    assert torch.equal(ta.sampler.n_id[:int(ta.sampler.sizes[0])],
                       tb.sampler.n_id[:int(tb.sampler.sizes[0])])
    assert float((ta.pflat - tb.pflat).abs().max()) <= 1e-3


def test_trainer_epoch_wraps_and_counts():
    """steps_per_epoch = ceil(ceil(n/B) / W); the last batch of an epoch is partial."""
    d = _mag(0.002, seed=4)
    tr, _ = _setup_trainer(d, d["model"](), batch=100, sizes=(4, 3))
    n = d["n_paper"]
    steps = tr.steps_per_epoch()
    assert steps == -(-n // 100)
    seen = []
    for _ in range(steps):
        tr.step()
        seen.append(tr.sampler.n_id[:int(tr.sampler.sizes[0])].cpu())
    allt = torch.cat(seen)
    assert sorted(allt.tolist()) == list(range(n))       # one epoch covers every target once
    assert int(tr.sampler.sizes[0]) == n - 100 * (steps - 1)


def test_dp_union_gradient_equals_mean_of_halves():
    """per-target samples are keyed on (hop seed, node): two half-batches sampled with the batch
    index of their union see the same neighbourhoods, so mean(grad(half_a), grad(half_b)) equals
    grad(union) -- what the flat-bucket all-reduce computes across two ranks."""
    from regnn_hip import mag
    from regnn_hip.sampler import NeighborSampler
    d = _mag(0.003, seed=5)
    smp = NeighborSampler(d["rg"], torch.arange(d["n_paper"], device=DEV), [8, 5], batch_size=128,
                          shuffle=False, seed=11)
    union = torch.randperm(d["n_paper"], generator=torch.Generator().manual_seed(0))[:128].to(DEV)
    grads = []
    for part in (union, union[:64], union[64:]):
        m = d["model"]()
        m.train()
        opt = torch.optim.SGD(m.parameters(), lr=0.0)
        mag.train_step(m, opt, smp.sample(part, 4), d["x_dict"], d["edge_type"], d["node_type"],
                       d["local"], d["y"], 1)
        grads.append({n: p.grad.double().cpu() for n, p in m.named_parameters()
                      if p.grad is not None})        # REGNN.norm: declared, unused
    for n in grads[0]:
        mean = 0.5 * (grads[1][n] + grads[2][n])
        err = (mean - grads[0][n]).abs().max().item()
        scale = max(1e-3, grads[0][n].abs().max().item())
        assert err <= 2e-6 * scale, f"{n}: {err:.3e} (scale {scale:.3e})"


def test_ns_step_mag10_scale():
    """BASELINE config 5 at its own size: mag_like(10) (19.4 M nodes, 422 M raw edges), batch 512,
    fan-out [25, 20]: one device-engine step; sampled targets against the oracle spec (sampled
    rows re-derived with sampler_oracle.sample_row from the CSR rows), count = min(deg, k),
    unique n_id, and block aggregation rows against fp64 sums."""
    from regnn_hip import ops
    d = _mag(10.0, seed=0, F=128, hidden=64, classes=349)
    rg = d["rg"]
    model = d["model"]()
    model.train()
    from regnn_hip import ns
    old_mode, old_str = ns.LEAN_LAST_HOP["mode"], ns.STRIDED["mode"]
    ns.LEAN_LAST_HOP["mode"] = "off"             # this test inspects the outermost n_id
    ns.STRIDED["mode"] = "off"                   # and the CSR blocks
    try:
        tr, _ = _setup_trainer(d, model, batch=512, sizes=(25, 20), seed=123)
    finally:
        ns.LEAN_LAST_HOP["mode"], ns.STRIDED["mode"] = old_mode, old_str
    tr.step()
    torch.cuda.synchronize()
    assert np.isfinite(float(tr.loss))
    s = tr.sampler
    sz = s.sizes.cpu().tolist()
    n_id = s.n_id[:sz[2]].cpu().numpy()
    assert np.unique(n_id).size == n_id.size
    ptr_d = rg.csr_ptr
    st = s.state.cpu().numpy()
    from regnn_hip.sampler import hop_seed
    rng = np.random.default_rng(0)
    for h, k in enumerate((25, 20)):
        blk = s.blocks[h]
        n_dst, E = sz[h], sz[8 + h]
        bp = blk.csr_ptr[:n_dst + 1].cpu().numpy()
        tgt = n_id[:n_dst]
        deg = (ptr_d[1:] - ptr_d[:-1]).cpu().numpy()[tgt]
        assert np.all(np.diff(bp) == np.minimum(deg, k) + 1)
        assert E == bp[-1]
        pos = blk.pos[:E].cpu().numpy()
        idx_l = blk.csr_idx[:E].cpu().numpy()
        seed = hop_seed(int(st[0]) & ((1 << 64) - 1), int(st[1]), int(st[3]), h)
        for v in rng.choice(n_dst, size=24, replace=False):
            t = int(tgt[v])
            a, b = int(ptr_d[t]), int(ptr_d[t + 1])
            row_idx = rg.csr_idx[a:b].cpu().numpy()
            # the oracle's row sampler (keyed on the global target id) on this CSR row
            want_src, want_pos = _sample_row_global(row_idx, t, k, seed, a)
            got_pos = pos[bp[v]:bp[v + 1] - 1]
            assert got_pos.tolist() == want_pos
            assert n_id[idx_l[bp[v]:bp[v + 1] - 1]].tolist() == want_src
    # layer-0 block aggregation rows (the outermost hop) against fp64 sums
    blk = s.blocks[1]
    n_dst = sz[1]
    x = torch.randn(s.caps[2], 64, device=DEV)
    tab = torch.linspace(-0.3, 1.2, 11, device=DEV)
    bias = torch.randn(64, device=DEV)
    y = ops.ns_spmm(blk, x, tab, bias).cpu().double().numpy()
    xd = x.cpu().double().numpy()
    bp = blk.csr_ptr.cpu().numpy()
    ix, rl = blk.csr_idx.cpu().numpy(), blk.rel.cpu().numpy()
    tb = tab.cpu().double().numpy()
    for v in rng.choice(n_dst, size=200, replace=False):
        e = np.arange(bp[v], bp[v + 1])
        want = (tb[rl[e]][:, None] * xd[ix[e]]).sum(0) / e.size + bias.cpu().double().numpy()
        assert np.allclose(y[v], want, rtol=1e-5, atol=1e-5)


def test_ns_step_mag10_fused_matches_module_path():
    """the benchmarked mode at its own size: mag_like(10), batch 512, fan-out
    [25, 20], K = 128, hidden 64, 349 classes, relation slots on and the meta-only last hop.
    The fused step's loss and every parameter gradient equal the mag.REGNN autograd path's (pinned
    to the reference REGNN by tests/test_gpu_regnn_golden.py) on the same sampled batch at 1e-5,
    dropout off."""
    d = _mag(10.0, seed=0, F=128, hidden=64, classes=349)
    m_mod, m_fus = d["model"](3), d["model"](3)
    m_mod.train(); m_fus.train()
    tr_f, _ = _setup_trainer(d, m_fus, batch=512, sizes=(25, 20), seed=123)
    assert tr_f.fused is not None and tr_f.fused.P.rel_slots == 1
    assert tr_f.sampler.meta_only[1]
    tr_m, _ = _setup_trainer(d, m_mod, batch=512, sizes=(25, 20), seed=123)
    tr_m.fused = None
    tr_f._forward_backward()
    tr_m._forward_backward()
    torch.cuda.synchronize()
    assert torch.equal(tr_m.sampler.sizes[8:10], tr_f.sampler.sizes[8:10])
    assert int(tr_f.sampler.sizes[9]) > 100_000                 # the full-size layer-0 block
    lm, lf = float(tr_m.loss), float(tr_f.loss)
    assert abs(lm - lf) <= 1e-5 * max(1.0, abs(lm)), (lm, lf)
    gm = dict(m_mod.named_parameters())
    for n, p in m_fus.named_parameters():
        ok, err = G.close(p.grad.cpu().numpy(), gm[n].grad.cpu().numpy().astype(np.float64), 1e-5)
        assert ok, f"{n}: rel err {err:.3e}"


def _sample_row_global(row_idx, t, k, seed, base):
    d = row_idx.size
    if d <= k:
        return row_idx.tolist(), [base + q for q in range(d)]
    chosen = []
    for j in range(d - k, d):
        pos = (SO.sample_hash(seed, t, j) * (j + 1)) >> 32
        chosen.append(j if pos in chosen else pos)
    chosen.sort()
    return [int(row_idx[p]) for p in chosen], [base + p for p in chosen]


def _nsm_seed(st, layer):
    """the fused step's dropout seed of `layer` (include/regnn_hip.h, regnn_nsm_step): seed
    word, epoch and global batch of the step's sampler state."""
    from regnn_hip.sampler import _mix
    M = (1 << 64) - 1
    return _mix((st[0] & M) ^ _mix(((st[1] << 40) ^ (st[3] << 8) ^ (layer + 0x51ED27)) & M))


@pytest.mark.parametrize("rel_slots", ["auto", "off"])
@pytest.mark.parametrize("dropout", [0.0, 0.5])
def test_fused_step_matches_module_path(monkeypatch, dropout, rel_slots):
    """regnn_nsm_step (the model's forward / nll / backward in eight launches) against the
    mag.REGNN autograd path on the same sampled batch: loss and every parameter gradient at
    1e-5, with layer 0's relation-table gradient from the per-source-type slot sums (the
    ogbn-mag schema allows it) and from the edge pass. With dropout the module path gets the
    fused step's hash masks (oracle.dropout_mask of the documented per-layer seed) in place of
    torch's RNG."""
    from oracle import regnn_oracle as O
    from regnn_hip import ns
    monkeypatch.setitem(ns.REL_SLOTS, "mode", rel_slots)
    d = _mag(0.003, seed=6, F=128, hidden=64, classes=37, dropout=dropout)
    m_mod, m_fus = d["model"](1), d["model"](1)
    m_mod.train(); m_fus.train()
    tr_m, _ = _setup_trainer(d, m_mod, batch=96, sizes=(7, 5))
    tr_m.fused = None                                   # the module (autograd) path
    tr_f, _ = _setup_trainer(d, m_fus, batch=96, sizes=(7, 5))
    assert tr_f.fused is not None
    assert tr_f.fused.P.rel_slots == (1 if rel_slots == "auto" else 0)
    tr_f._forward_backward()
    torch.cuda.synchronize()
    st = tr_f.sampler.state.cpu().tolist()
    calls = []
    if dropout > 0:
        keep16 = int(round((1 - dropout) * 65536))

        def hash_dropout(x, p=0.5, training=True, inplace=False):
            layer = len(calls)
            calls.append(layer)
            seed = _nsm_seed(st, layer)
            mask = O.dropout_mask(seed, x.shape[0], x.shape[1], 4, keep16)
            return x * torch.from_numpy(mask).to(x.device, x.dtype) / (keep16 / 65536)
        monkeypatch.setattr(torch.nn.functional, "dropout", hash_dropout)
    tr_m._forward_backward()
    torch.cuda.synchronize()
    if dropout > 0:
        assert calls == [0, 1]
    # the fused trainer's last hop is meta-only: n_id agrees up to the layer-0 targets, the
    # blocks' sizes everywhere
    n0 = int(tr_f.sampler.sizes[1])
    assert torch.equal(tr_m.sampler.sizes[8:10], tr_f.sampler.sizes[8:10])
    assert torch.equal(tr_m.sampler.n_id[:n0], tr_f.sampler.n_id[:n0])
    lm, lf = float(tr_m.loss), float(tr_f.loss)
    assert abs(lm - lf) <= 1e-5 * max(1.0, abs(lm)), (lm, lf)
    gm = dict(m_mod.named_parameters())
    for n, p in m_fus.named_parameters():
        ok, err = G.close(p.grad.cpu().numpy(), gm[n].grad.cpu().numpy().astype(np.float64), 1e-5)
        assert ok, f"{n}: rel err {err:.3e}"


def test_fused_step_large_batch_takes_composed_form():
    """a batch whose hop-0 block exceeds the transposed index (1300 x 26 = 33,800 >
    32,768 edges at fan-out 25) runs regnn_nsm_step's composed-map form: the library's slab size
    and step follow the caller's two_layer flag, and loss / gradients match the module path."""
    d = _mag(0.003, seed=6, F=128, hidden=64, classes=37, dropout=0.0)
    m_mod, m_fus = d["model"](1), d["model"](1)
    tr_m, _ = _setup_trainer(d, m_mod, batch=1300, sizes=(25, 20))
    tr_m.fused = None
    tr_f, _ = _setup_trainer(d, m_fus, batch=1300, sizes=(25, 20))
    assert tr_f.fused is not None and not tr_f.fused.two_layer
    assert tr_f.fused.P.two_layer == 0
    tr_f._forward_backward()
    tr_m._forward_backward()
    torch.cuda.synchronize()
    lm, lf = float(tr_m.loss), float(tr_f.loss)
    assert abs(lm - lf) <= 1e-5 * max(1.0, abs(lm)), (lm, lf)
    gm = dict(m_mod.named_parameters())
    for n, p in m_fus.named_parameters():
        ok, err = G.close(p.grad.cpu().numpy(), gm[n].grad.cpu().numpy().astype(np.float64), 1e-5)
        assert ok, f"{n}: rel err {err:.3e}"


def test_fused_step_fixed_point_overflow_reads_nan():
    """layer 1's transposed pass sums 2^-40 fixed-point terms; a term past the
    documented range (2^8) flags the step, whose loss then reads NaN (instead of a silently
    wrapped gradient), and the next in-range step is clean again."""
    d = _mag(0.003, seed=6, F=128, hidden=64, classes=37, dropout=0.0)
    m = d["model"](1)
    m.train()
    tr, _ = _setup_trainer(d, m, batch=96, sizes=(7, 5), lr=0.0)
    assert tr.fused is not None and tr.fused.two_layer
    tr._forward_backward()
    torch.cuda.synchronize()
    assert np.isfinite(float(tr.loss))
    with torch.no_grad():                      # GH rows scale with out_lin.weight (layer 1's
        w_out = m.out_lin.weight.clone()       # LayerNorm cancels a conv weight scale)
        m.out_lin.weight.mul_(1e7)
    tr._forward_backward()
    torch.cuda.synchronize()
    assert np.isnan(float(tr.loss))
    with torch.no_grad():
        m.out_lin.weight.copy_(w_out)
    tr._forward_backward()
    torch.cuda.synchronize()
    assert np.isfinite(float(tr.loss))


@pytest.mark.parametrize("flat_adam", [False, True])
def test_fused_step_graph_replay_tracks_eager(flat_adam):
    """the fused step captured in a HIP graph: losses equal the eager twin's step by step
    (torch Adam(capturable) or the one-launch FlatAdam)."""
    from regnn_hip.ns import NSTrainer
    d = _mag(0.003, seed=7, F=128, hidden=64, classes=11, dropout=0.3)

    def make():
        if not flat_adam:
            return _setup_trainer(d, d["model"](4), batch=128, sizes=(10, 5))[0]
        return NSTrainer(d["model"](4), None, d["rg"], [10, 5], 128,
                         torch.arange(d["n_paper"], device=DEV), d["x_dict"], d["edge_type"],
                         d["node_type"], d["local"], d["y"], 7, seed=3, adam=dict(lr=1e-2))
    tr_e, tr_g = make(), make()
    assert tr_e.fused is not None and tr_g.fused is not None
    tr_g.capture(warmup=2)                             # warm-up steps undone by capture()
    le, lg = [], []
    for _ in range(5):
        tr_e.step()
        le.append(float(tr_e.loss))
        tr_g.replay()
        lg.append(float(tr_g.loss))
    assert np.all(np.isfinite(lg))
    assert np.allclose(le, lg, rtol=1e-4, atol=1e-5), (le, lg)


@pytest.mark.parametrize("pre", ["on", "off"])
@pytest.mark.parametrize("odd", [True, False])
@pytest.mark.parametrize("wd,gs", [(0.0, 1.0), (1e-3, 1.0), (0.0, 0.125)])
def test_flat_adam_matches_torch_adam(wd, gs, odd, pre, monkeypatch):
    """regnn_adam_flat (the NS trainer's one-launch optimizer) against torch.optim.Adam over
    the same gradients for 4 steps, with and without weight decay; grad_scale 1/8 (the mean of
    an 8-rank SUM all-reduce) against torch's Adam on the divided gradient. odd: a bucket of
    30603 elements (the scalar kernel); else 30604 (the float4 kernel). pre: the step count
    advanced by a stream op before the launch (no ticket) or by the kernel's last block."""
    from regnn_hip import ns
    from regnn_hip.ns import FlatAdam
    monkeypatch.setitem(ns.ADAM_PRE_STEP, "mode", pre)
    g = torch.Generator(device=DEV).manual_seed(5)
    shapes = [(64, 128), (64,), (11,) if odd else (12,), (349, 64)]
    ref = [torch.randn(s, generator=g, device=DEV).requires_grad_(True) for s in shapes]
    opt = torch.optim.Adam(ref, lr=1e-2, weight_decay=wd)
    pflat = torch.cat([p.detach().reshape(-1) for p in ref]).clone()
    gflat = torch.zeros_like(pflat)
    fa = FlatAdam(pflat, gflat, lr=1e-2, weight_decay=wd)
    fa.grad_scale = gs
    for _ in range(4):
        grads = [torch.randn(s, generator=g, device=DEV) for s in shapes]
        for p, gr in zip(ref, grads):
            p.grad = gr * gs
        gflat.copy_(torch.cat([gr.reshape(-1) for gr in grads]))
        opt.step()
        fa.step()
    torch.cuda.synchronize()
    want = torch.cat([p.detach().reshape(-1) for p in ref])
    assert int(fa.step_count) == 4
    assert torch.allclose(pflat, want, rtol=1e-6, atol=1e-7), (pflat - want).abs().max()


def test_meta_only_last_hop_matches_full_hop():
    """regnn_ns_hop meta_only (the fused trainer's last hop: no dedup, no n_id append) writes
    the same block pointers, relation ids, CSR positions, 1/in-counts and per-edge source type /
    table row as the full hop, and the fused step's loss and every gradient are bitwise equal
    (the two-layer step's reductions are fixed-order or exact)."""
    from regnn_hip import ns
    d = _mag(0.003, seed=4, F=128, hidden=64, classes=17, dropout=0.5)
    outs = []
    for mode in ("off", "on"):
        ns.LEAN_LAST_HOP["mode"] = mode
        ns.STRIDED["mode"] = "off"               # the CSR blocks are compared
        try:
            model = d["model"](2)
            model.train()
            tr, _ = _setup_trainer(d, model, batch=80, sizes=(6, 5))
        finally:
            ns.LEAN_LAST_HOP["mode"] = "on"
            ns.STRIDED["mode"] = "on"
        assert tr.fused is not None
        tr._forward_backward()
        torch.cuda.synchronize()
        s = tr.sampler
        sz = s.sizes.cpu().tolist()
        blk = s.blocks[1]
        E, n1 = sz[9], sz[1]
        et, eo = s.edge_meta[1]
        outs.append(dict(sz=sz[8:10] + sz[:2], ptr=blk.csr_ptr[:n1 + 1].clone(),
                         rel=blk.rel[:E].clone(), pos=blk.pos[:E].clone(), inv=blk.inv[:n1].clone(),
                         et=et[:E].clone(), eo=eo[:E].clone(), loss=tr.loss.clone(),
                         grads=[p.grad.clone() for p in model.parameters()]))
    a, b = outs
    assert a["sz"] == b["sz"]
    for k in ("ptr", "rel", "pos", "inv", "et", "eo", "loss"):
        assert torch.equal(a[k], b[k]), k
    for ga, gb in zip(a["grads"], b["grads"]):
        assert torch.equal(ga, gb), (ga - gb).abs().max()


@pytest.mark.parametrize("ahead", [1, 4])
def test_run_steps_pair_graph_matches_single_replays(monkeypatch, ahead):
    """run_steps (ahead 1: runs of 4 / 2 steps as one multi-step graph replay; ahead 4: 4-step
    graphs whose sampler fills the other four slots) trains the same batches to the same losses
    and bitwise the same parameters as one-step replays, across an epoch boundary (the
    two-layer step is bitwise reproducible: VERDICT r2 item 8)."""
    d = _mag(0.002, seed=8, F=128, hidden=64, classes=13, dropout=0.4)
    from regnn_hip import ns
    from regnn_hip.ns import NSTrainer
    monkeypatch.setitem(ns.AHEAD, "steps", ahead)

    def make():
        return NSTrainer(d["model"](5), None, d["rg"], [6, 4], 100,
                         torch.arange(d["n_paper"], device=DEV), d["x_dict"], d["edge_type"],
                         d["node_type"], d["local"], d["y"], 7, seed=9, adam=dict(lr=1e-2))
    ta, tb = make(), make()
    ta.capture(warmup=1)
    tb.capture(warmup=1)
    assert ta.ahead == ahead and len(ta.slots) == 2 * ahead
    assert sorted(ta.graph_groups) == ([2, 4] if ahead == 1 else
                                       [(m, c) for m in (2, 4) for c in range(8)])
    for k in (4, 3, 2, 7):              # odd counts end on a single replay
        ta.run_steps(k)
        for _ in range(k):
            tb.replay()
        torch.cuda.synchronize()
        assert ta.cur == tb.cur and ta._trained == tb._trained
        assert float(ta.loss) == float(tb.loss)
        assert torch.equal(ta.sampler.n_id[:int(ta.sampler.sizes[0])],
                           tb.sampler.n_id[:int(tb.sampler.sizes[0])])
        assert torch.equal(ta.pflat, tb.pflat), (ta.pflat - tb.pflat).abs().max()
    ta.set_epoch(1)
    tb.set_epoch(1)
    ta.run_steps(2)
    tb.replay(); tb.replay()
    torch.cuda.synchronize()
    assert torch.equal(ta.sampler.n_id[:int(ta.sampler.sizes[0])],
                       tb.sampler.n_id[:int(tb.sampler.sizes[0])])
    assert float(ta.loss) == float(tb.loss)
    assert torch.equal(ta.pflat, tb.pflat), (ta.pflat - tb.pflat).abs().max()


@pytest.mark.parametrize("rel_slots", ["auto", "off"])
def test_two_layer_step_bitwise_reproducible(monkeypatch, rel_slots):
    """the two-layer fused step run twice on the same batch (eager, dropout on): loss and every
    gradient bitwise equal (fixed-order reductions; layer 1's transposed aggregation as exact
    fixed-point integer sums) -- VERDICT r2 item 8."""
    from regnn_hip import ns
    monkeypatch.setitem(ns.REL_SLOTS, "mode", rel_slots)
    d = _mag(0.003, seed=9, F=128, hidden=64, classes=29, dropout=0.5)
    outs = []
    for _ in range(2):
        m = d["model"](4)
        m.train()
        tr, _ = _setup_trainer(d, m, batch=128, sizes=(10, 6))
        assert tr.fused is not None and tr.fused.two_layer
        assert tr.fused.kernels()[:4] == ["agg0", "head", "gather", "bwd0"]
        tr._forward_backward()
        torch.cuda.synchronize()
        outs.append((float(tr.loss), [p.grad.clone() for p in m.parameters()]))
    assert outs[0][0] == outs[1][0]
    for ga, gb in zip(outs[0][1], outs[1][1]):
        assert torch.equal(ga, gb)


def test_pre_sums_match_in_kernel_gather(monkeypatch):
    """layer 0's per-type input sums formed on the sampler stream (regnn_ns_hop_typed_sums,
    PRE_SUMS on) against agg0's own gather (off) on the same batch: the sampler adds each row's
    entries in slot order as agg0 does, so sums, counts, self rows, slot relations, the loss and
    every gradient are bitwise equal."""
    from regnn_hip import ns
    d = _mag(0.003, seed=9, F=128, hidden=64, classes=29, dropout=0.5)
    res = {}
    for mode in ("on", "off"):
        monkeypatch.setitem(ns.PRE_SUMS, "mode", mode)
        m = d["model"](4)
        m.train()
        tr, _ = _setup_trainer(d, m, batch=128, sizes=(10, 6))
        assert bool(tr.fused.W.pre_sums) == (mode == "on")
        tr._forward_backward()
        torch.cuda.synchronize()
        fs = tr.fused_slots[tr._trained] if tr.pipelined else tr.fused
        n1 = int(tr.sampler.sizes[1])
        W = fs.W
        res[mode] = (float(tr.loss), [p.grad.clone() for p in m.parameters()],
                     [fs._buf(a)[:n1].clone() for a in (W.s_agg, W.s_w, W.u_self, W.u_rel)])
    (la, ga, ba), (lb, gb, bb) = res["on"], res["off"]
    for x, y in zip(ba, bb):
        assert torch.equal(x, y)
    assert la == lb
    for x, y in zip(ga, gb):
        assert torch.equal(x, y)


def test_fused_adam_equals_separate_adam(monkeypatch):
    """a one-rank FlatAdam trainer's optimizer inside the step's last launch (FUSED_ADAM on)
    gives the parameters, moments and step count of the separate regnn_adam_flat launch (the
    same arithmetic; 1e-6, the two kernels' instruction selection may differ) after several
    eager steps and graph replays."""
    from regnn_hip import ns
    from regnn_hip.ns import NSTrainer
    d = _mag(0.002, seed=8, F=128, hidden=64, classes=13, dropout=0.4)
    trs = []
    for mode in ("on", "off"):
        monkeypatch.setitem(ns.FUSED_ADAM, "mode", mode)
        trs.append(NSTrainer(d["model"](5), None, d["rg"], [6, 4], 100,
                             torch.arange(d["n_paper"], device=DEV), d["x_dict"], d["edge_type"],
                             d["node_type"], d["local"], d["y"], 7, seed=9,
                             adam=dict(lr=1e-2, weight_decay=1e-4)))
    a, b = trs
    assert a.adam_fused and not b.adam_fused
    assert a.fused.kernels()[-1] == "finalize+adam"
    for _ in range(3):
        a.step()
        b.step()
    a.capture(warmup=1)
    b.capture(warmup=1)
    a.run_steps(5)
    b.run_steps(5)
    torch.cuda.synchronize()
    assert abs(float(a.loss) - float(b.loss)) <= 1e-5 * max(1.0, abs(float(b.loss)))
    # REGNN.norm (declared, never read by the forward: no gradient) is stepped by the bucket-wide
    # regnn_adam_flat (weight decay moves it) but, as torch.optim.Adam skips a parameter without
    # a gradient, not by the fused optimizer
    keep = torch.ones_like(a.pflat, dtype=torch.bool)
    for (name, p), o in zip(a.model.named_parameters(), a.offsets):
        if name.startswith("norm."):
            keep[o:o + p.numel()] = False
    for x, y in ((a.pflat, b.pflat), (a.opt.m, b.opt.m), (a.opt.v, b.opt.v)):
        x, y = x[keep], y[keep]
        assert torch.allclose(x, y, rtol=1e-5, atol=1e-6), (x.double() - y.double()).abs().max()
    assert int(a.opt.step_count) == int(b.opt.step_count) == 8


def test_block_transposed_index():
    """regnn_ns_hop's transposed index of a block (csc_ptr / csc_ent): per local source u, the
    multiset of (target row << 8 | relation) over the block edges whose source is u, and the
    block's per-edge target rows (blk_row)."""
    from regnn_hip.graph import RelGraph
    from regnn_hip.ns import DeviceSampler
    rng = np.random.default_rng(12)
    N, E = 5000, 80000
    dst = np.minimum((rng.pareto(1.1, E) * 4).astype(np.int64), N - 1)
    src = np.where(rng.random(E) < 0.6, rng.integers(0, 3, E), rng.integers(0, N, E))  # 3 hubs
    rg = RelGraph(src, dst, N, DEV)
    ds = DeviceSampler(rg, [12, 5], 150, etype=torch.from_numpy(rng.integers(0, 7, E)),
                       ntype=torch.from_numpy(rng.integers(0, 4, N)), num_edge_types=7)
    _, cptr, cent, clong = ds.enable_csc(0)
    ds.set_seed(5, 0, 1)
    ds.set_targets(torch.from_numpy(rng.permutation(N)[:150]).to(DEV))
    ds.run_hops()
    sz = ds.sizes.cpu().tolist()
    n_dst, n_src, Eb = sz[0], sz[1], sz[8]
    blk = ds.blocks[0]
    ptr = blk.csr_ptr[:n_dst + 1].cpu().numpy()
    idx = blk.csr_idx[:Eb].cpu().numpy()
    rel = blk.rel[:Eb].cpu().numpy().astype(np.int64)
    row = blk.row[:Eb].cpu().numpy()
    assert np.array_equal(row, np.repeat(np.arange(n_dst), np.diff(ptr)))
    cp = cptr[:n_src + 1].cpu().numpy()
    ce = cent[:Eb].cpu().numpy().astype(np.int64)
    assert cp[0] == 0 and cp[-1] == Eb and np.all(np.diff(cp) >= 1)   # every source has an edge
    want = [[] for _ in range(n_src)]
    for bp in range(Eb):
        want[idx[bp]].append((int(row[bp]) << 8) | int(rel[bp]))
    for u in range(n_src):
        assert sorted(ce[cp[u]:cp[u + 1]].tolist()) == sorted(want[u]), u
    cl = clong.cpu().numpy()
    longs = np.nonzero(np.diff(cp) > 16)[0]
    assert cl[0] == longs.size and longs.size > 0 and np.array_equal(cl[1:1 + cl[0]], longs)


def test_transposed_index_after_csr_batches():
    """batches in the CSR layout (exact_adjs, the module path) and in the
    strided layout alternating on one sampler. The strided index's control words (ticket,
    published stamp, error word) lie past the CSR de-duplication's tile words, so a tile count a
    CSR batch leaves behind cannot pass for the publish: here the old publish word (tiles[1]) is
    even set to the coming hop's stamp before each strided batch. Every batch's index equals the
    block's transposed multiset and the error word stays 0."""
    from regnn_hip.graph import RelGraph
    from regnn_hip.ns import DeviceSampler
    rng = np.random.default_rng(13)
    N, E = 5000, 80000
    dst = np.minimum((rng.pareto(1.1, E) * 4).astype(np.int64), N - 1)
    src = np.where(rng.random(E) < 0.6, rng.integers(0, 3, E), rng.integers(0, N, E))
    rg = RelGraph(src, dst, N, DEV)
    ds = DeviceSampler(rg, [12, 5], 150, etype=torch.from_numpy(rng.integers(0, 7, E)),
                       ntype=torch.from_numpy(rng.integers(0, 4, N)), num_edge_types=7)
    _, cptr, cent, clong = ds.enable_csc(0)
    assert ds.hop_bufs[0]["tiles"].numel() >= 2 + 4     # two flag tiles: tiles[1] a tile word
    for it, strided in enumerate([False, True, False, True, True]):
        ds.set_seed(5, 0, it)
        ds.set_targets(torch.from_numpy(rng.permutation(N)[:150]).to(DEV))
        if strided:
            ds.hop_bufs[0]["tiles"][1] = int(ds.state[4].item()) * 8 + 1   # hop 0's stamp
        ds.run_hops(strided=strided)
        sz = ds.sizes.cpu().tolist()
        n_dst, n_src = sz[0], sz[1]
        blk = ds.blocks[0]
        if strided:
            S = ds.sizes_k[0] + 1
            cnt = ds.hop_bufs[0]["scnt"][:n_dst].cpu().numpy()
            pos = np.concatenate([np.arange(i * S, i * S + cnt[i] + 1) for i in range(n_dst)])
        else:
            pos = np.arange(int(blk.csr_ptr[n_dst].item()))
        pos_t = torch.from_numpy(pos).to(DEV)
        idx = blk.csr_idx[pos_t].cpu().numpy()
        rel = blk.rel[pos_t].cpu().numpy().astype(np.int64)
        row = blk.row[pos_t].cpu().numpy()
        Eb = pos.size
        assert sz[8] == Eb
        cp = cptr[:n_src + 1].cpu().numpy()
        ce = cent[:Eb].cpu().numpy().astype(np.int64)
        assert cp[0] == 0 and cp[-1] == Eb and np.all(np.diff(cp) >= 1), (it, strided)
        want = [[] for _ in range(n_src)]
        for bp in range(Eb):
            want[idx[bp]].append((int(row[bp]) << 8) | int(rel[bp]))
        for u in range(n_src):
            assert sorted(ce[cp[u]:cp[u + 1]].tolist()) == sorted(want[u]), (it, strided, u)
        assert not any(ds.index_errors().cpu().tolist())
    ds.check_index()


@pytest.mark.parametrize("half_waves,csc_fuse", [("0", "on"), ("1", "on"), ("0", "off")])
def test_strided_blocks_match_csr(monkeypatch, half_waves, csc_fuse):
    """regnn_ns_hop strided (the fused engine's fixed-stride blocks: sampling and placement in one
    launch) against the CSR layout on the same batches: the same n_id, sizes, per-row edges
    (local source, relation, CSR position, target row; the meta-only hop's source type / table
    row), 1/in-counts and transposed index; and the two-layer fused step's loss and gradients
    bitwise equal over both layouts. half_waves "1": the strided sampler with two targets per
    wave (fan-outs 9 and 7 fit 32 lanes)."""
    from regnn_hip import ns
    monkeypatch.setenv("REGNN_NS_HALF_WAVES", half_waves)
    # "on": hop 0's transposed index built by extra workgroups of hop 1's sums launch; "off": its
    # own launch after the de-duplication
    monkeypatch.setitem(ns.CSC_FUSE, "mode", csc_fuse)
    d = _mag(0.003, seed=10, F=128, hidden=64, classes=19, dropout=0.5)
    trs, models = [], []
    for mode in ("off", "on"):
        monkeypatch.setitem(ns.STRIDED, "mode", mode)
        m = d["model"](6)
        m.train()
        tr, _ = _setup_trainer(d, m, batch=120, sizes=(9, 7))
        assert tr.sampler.strided == (mode == "on")
        trs.append(tr)
        models.append(m)
    a, b = trs                                   # CSR, strided
    for _ in range(2):
        a._forward_backward()
        b._forward_backward()
        torch.cuda.synchronize()
        sa, sb = a.sampler, b.sampler
        assert torch.equal(sa.sizes, sb.sizes)
        n1 = int(sa.sizes[1])
        assert torch.equal(sa.n_id[:n1], sb.n_id[:n1])
        for h, k in enumerate(sa.sizes_k):
            S, n_dst = k + 1, int(sa.sizes[h])
            ba, bb = sa.blocks[h], sb.blocks[h]
            ptr = ba.csr_ptr[:n_dst + 1].cpu().numpy()
            cnt = sb.hop_bufs[h]["scnt"][:n_dst].cpu().numpy()
            assert np.array_equal(np.diff(ptr), cnt + 1)
            assert torch.equal(ba.inv[:n_dst], bb.inv[:n_dst])
            pos = np.concatenate([np.arange(i * S, i * S + cnt[i] + 1) for i in range(n_dst)])
            pos_t = torch.from_numpy(pos).to(DEV)
            E = int(ptr[-1])
            assert torch.equal(ba.rel[:E], bb.rel[pos_t])
            if sa.meta_only[h]:
                for ma, mb in zip(sa.edge_meta[h], sb.edge_meta[h]):
                    assert torch.equal(ma[:E], mb[pos_t])
            else:
                for xa, xb in ((ba.csr_idx, bb.csr_idx), (ba.pos, bb.pos), (ba.row, bb.row)):
                    assert torch.equal(xa[:E], xb[pos_t])
        ca, cb = sa.csc[0], sb.csc[0]
        n0 = int(sa.sizes[1])
        assert torch.equal(ca[1][:n0 + 1], cb[1][:n0 + 1])          # csc_ptr
        assert torch.equal(ca[3][:1], cb[3][:1])                      # hub count
        E0 = int(sa.sizes[8])
        assert torch.equal(torch.sort(ca[2][:E0])[0], torch.sort(cb[2][:E0])[0])
        assert float(a.loss) == float(b.loss)
        for pa, pb in zip(models[0].parameters(), models[1].parameters()):
            assert torch.equal(pa.grad, pb.grad)
