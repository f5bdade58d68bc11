"""GPU parity of the ogbn-mag path: mag REGCNConv vs golden vectors from mag/regnn_layers.py, and the
GPU neighbour sampler vs the sampler oracle (bit-exact)."""
import numpy as np
import pytest
import torch

import _golden as G
from oracle import sampler_oracle as SO

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL = 1e-5


def _check(tag, got, want, tol=TOL):
    got = got.detach().float().cpu().numpy()
    ok, err = G.close(got, want, tol)
    assert ok, f"{tag}: rel err {err:.3e}"


@pytest.mark.parametrize("name", G.names("mag_regcnconv_"))
def test_mag_regcnconv(name):
    from regnn_hip.mag import REGCNConv
    d = G.load(name)
    m = d["meta"]
    sm = bool(m.get("use_softmax", False))
    conv = REGCNConv(64, 64, m["num_node_types"], m["num_edge_types"], m["scaling_factor"],
                     use_softmax=sm, residual=m["residual"], use_norm=m["use_norm"],
                     self_loop_type=2)
    P = G.sub(d, "p_", np.float32)
    assert {n for n, _ in conv.named_parameters()} == set(P)
    with torch.no_grad():
        for n, p in conv.named_parameters():
            p.copy_(torch.from_numpy(P[n]))
    conv = conv.to(DEV)
    x = torch.from_numpy(d["x"]).to(DEV).requires_grad_(True)
    ei = torch.from_numpy(np.stack([d["src"], d["dst"]])).to(DEV)
    res = conv((x, x[:m["n_dst"]]), ei, torch.from_numpy(d["edge_type"]).to(DEV),
               torch.from_numpy(d["target_node_type"]).to(DEV), return_weights=sm)
    out = res[0] if sm else res
    out.backward(torch.from_numpy(d["gout"]).to(DEV))
    _check("out", out, d["out"])
    if sm:           # the reference computes the softmax ew but propagates the raw weights
        _check("ew", res[1], d["ew"])
    _check("grad_x", x.grad, d["grad_x"])
    for k, v in G.sub(d, "grad_").items():
        if k != "x":
            _check(k, dict(conv.named_parameters())[k].grad, v)


@pytest.mark.parametrize("name", G.names("mag_regatconv_") + G.names("mag_regatv2conv_"))
def test_mag_regatconv(name):
    """mag REGATConv / REGATv2Conv (global-max softmax) vs golden vectors."""
    from regnn_hip import mag
    d = G.load(name)
    m = d["meta"]
    cls = mag.REGATv2Conv if "v2" in m["layer"] else mag.REGATConv
    H, C = m["heads"], m["out_channels"]
    conv = cls(H * C, C, m["num_node_types"], m["num_edge_types"], heads=H,
               scaling_factor=m["scaling_factor"], residual=m["residual"],
               use_norm=m["use_norm"], self_loop_type=2)
    P = G.sub(d, "p_", np.float32)
    assert {n for n, _ in conv.named_parameters()} == set(P)
    with torch.no_grad():
        for n, p in conv.named_parameters():
            p.copy_(torch.from_numpy(P[n]))
    conv = conv.to(DEV)
    x = torch.from_numpy(d["x"]).to(DEV).requires_grad_(True)
    ei = torch.from_numpy(np.stack([d["src"], d["dst"]])).to(DEV)
    out = conv((x, x[:m["n_dst"]]), ei, torch.from_numpy(d["edge_type"]).to(DEV),
               torch.from_numpy(d["target_node_type"]).to(DEV))
    out.backward(torch.from_numpy(d["gout"]).to(DEV))
    _check("out", out, d["out"])
    _check("grad_x", x.grad, d["grad_x"])
    want = {k: v for k, v in G.sub(d, "grad_").items() if k != "x"}
    got = {n: p.grad for n, p in conv.named_parameters() if p.grad is not None}
    assert set(got) == set(want), set(got) ^ set(want)
    for k, v in want.items():
        _check(k, got[k], v)


@pytest.mark.parametrize("model", ["regat", "regatv2"])
def test_ns_gat_model_trains(model):
    """REGNN --model regat / regatv2 through the GPU sampler's fast blocks: finite gradients on
    every parameter and a falling loss over a few epochs."""
    from regnn_hip import mag, synth
    from regnn_hip.graph import RelGraph
    from regnn_hip.sampler import NeighborSampler
    gd = synth.mag_like(0.003, seed=1, device=DEV)
    keep = gd["rel"] <= 7
    rg = RelGraph(gd["src"][keep], gd["dst"][keep], gd["N"], DEV)
    edge_type = gd["rel"][keep].to(torch.int64) - 1
    node_type = gd["ntype"]
    offs = torch.tensor([gd["type_offsets"][t] for t in synth.NTYPES], device=DEV)
    local = torch.arange(gd["N"], device=DEV) - offs[node_type]
    feats = synth.type_features(gd["counts"], {t: 16 for t in synth.NTYPES}, seed=1, device=DEV)
    x_dict = {k: f for k, f in enumerate(feats)}
    torch.manual_seed(0)
    net = mag.REGNN(16, 8, 5, 2, 10.0, 0.0, {k: 16 for k in x_dict}, 7, use_norm="ln",
                    self_loop_type=2, model=model, heads=4).to(DEV)
    n_paper = gd["counts"]["paper"]
    y = torch.full((gd["N"], 1), -1, dtype=torch.int64, device=DEV)
    y[:n_paper, 0] = (torch.arange(n_paper, device=DEV) * 7) % 5
    smp = NeighborSampler(rg, torch.arange(n_paper, device=DEV), [10, 10], batch_size=256,
                          shuffle=True, seed=5)
    opt = torch.optim.Adam(net.parameters(), lr=1e-2)
    net.train()
    losses = []
    for epoch in range(3):
        smp.set_epoch(epoch)
        for batch in smp:
            losses.append(float(mag.train_step(net, opt, batch, x_dict, edge_type, node_type,
                                               local, y, 1)))
    assert all(np.isfinite(losses))
    assert np.mean(losses[-3:]) < np.mean(losses[:3])


def _power_graph(N=3000, E=40000, seed=0):
    rng = np.random.default_rng(seed)
    dst = np.minimum((rng.pareto(1.2, E) * 5).astype(np.int64), N - 1)
    src = rng.integers(0, N, E)
    return src, dst, N


@pytest.mark.parametrize("sizes", [[25, 20], [10, -1], [64]])
def test_sampler_bit_exact(sizes):
    from regnn_hip.graph import RelGraph
    from regnn_hip.sampler import NeighborSampler
    src, dst, N = _power_graph()
    rg = RelGraph(src, dst, N, DEV)
    ptr = rg.csr_ptr.cpu().numpy()
    idx = rg.csr_idx.cpu().numpy()
    eid = rg.csr_eid.cpu().numpy()
    smp = NeighborSampler(rg, torch.arange(N), sizes, batch_size=64, shuffle=False, seed=7)
    smp.set_epoch(3)
    for bi, batch in enumerate([torch.arange(0, 64), torch.arange(100, 164), torch.arange(5, 6)]):
        bs, n_id, adjs = smp.sample(batch.to(DEV), bi)
        rbs, rn_id, radjs = SO.neighbor_sample(ptr, idx, batch.tolist(), sizes, 7, epoch=3,
                                               batch_idx=bi)
        assert bs == rbs
        assert n_id.cpu().tolist() == rn_id
        adjs = adjs if isinstance(adjs, list) else [adjs]
        for a, (s, d_, e, size) in zip(adjs, radjs):
            ei, e_id, sz = a
            assert tuple(sz) == tuple(size)
            assert ei[0].cpu().tolist() == s
            assert ei[1].cpu().tolist() == d_
            assert e_id.cpu().tolist() == [int(eid[p]) for p in e]


def test_sampler_properties():
    """size-independent properties: no duplicate sampled neighbour per target, count = min(deg,k),
    every sampled edge exists, n_id unique, targets form the n_id prefix."""
    from regnn_hip.graph import RelGraph
    from regnn_hip.sampler import NeighborSampler
    src, dst, N = _power_graph(20000, 400000, seed=1)
    rg = RelGraph(src, dst, N, DEV)
    smp = NeighborSampler(rg, torch.arange(N), [25, 20], batch_size=512, shuffle=True, seed=1)
    bs, n_id, adjs = next(iter(smp))
    assert torch.unique(n_id).numel() == n_id.numel()
    deg = (rg.csr_ptr[1:] - rg.csr_ptr[:-1]).long()
    for (ei, e_id, (n_src, n_dst)), k in zip(adjs, [20, 25]):
        s, d_ = ei[0], ei[1]
        cnt = torch.bincount(d_, minlength=n_dst)
        assert torch.equal(cnt, deg[n_id[:n_dst]].clamp(max=k))
        assert torch.unique(e_id).numel() == e_id.numel()
        gs = torch.from_numpy(src).to(DEV)[e_id]
        gd = torch.from_numpy(dst).to(DEV)[e_id]
        assert torch.equal(gs, n_id[s]) and torch.equal(gd, n_id[d_])
