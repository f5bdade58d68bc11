"""GPU parity of the neighbour-sampled REGNN model (mag/regnn_ns.py:216-346) on a sampled batch:
GPU sampler -> group_input -> 2 x mag REGCNConv (+relu) -> out_lin -> log_softmax, forward and
parameter gradients against the fp64 oracle composed from oracle.regnn_oracle pieces (the conv
itself is pinned on golden vectors from mag/regnn_layers.py). Plus a short DP(world 1) training
run whose loss must fall."""
import numpy as np
import pytest
import torch

import _golden as G
from oracle import regnn_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _setup(scale=0.002, seed=0):
    from regnn_hip import mag, synth
    from regnn_hip.graph import RelGraph
    gd = synth.mag_like(scale, seed=seed, device=DEV)
    keep = gd["rel"] <= 7
    src, dst = gd["src"][keep], gd["dst"][keep]
    edge_type = gd["rel"][keep].to(torch.int64) - 1
    rg = RelGraph(src, dst, gd["N"], DEV)
    node_type = gd["ntype"]
    offs = torch.tensor([gd["type_offsets"][t] for t in synth.NTYPES], device=DEV)
    local = torch.arange(gd["N"], device=DEV) - offs[node_type]
    feats = synth.type_features(gd["counts"], {t: 16 for t in synth.NTYPES}, seed=1, device=DEV)
    x_dict = {k: f for k, f in enumerate(feats)}
    torch.manual_seed(0)
    model = mag.REGNN(16, 32, 5, 2, 10.0, 0.0, {k: 16 for k in x_dict}, 7, use_norm="ln",
                      self_loop_type=2).to(DEV)
    with torch.no_grad():          # relation weights off their constant init
        for conv in model.convs:
            conv.relation_weight.copy_(torch.rand(11, device=DEV) / 10.0)
            conv.bias.normal_(0, 0.1)
    return gd, rg, edge_type, node_type, local, x_dict, model


def test_ns_model_parity():
    from regnn_hip.sampler import NeighborSampler
    gd, rg, edge_type, node_type, local, x_dict, model = _setup()
    n_paper = gd["counts"]["paper"]
    smp = NeighborSampler(rg, torch.arange(n_paper, device=DEV), [6, 4], batch_size=64,
                          shuffle=True, seed=3)
    bs, n_id, adjs = next(iter(smp))
    model.eval()
    out = model(n_id, x_dict, adjs, edge_type, node_type, local)
    rng = np.random.default_rng(0)
    gout = rng.standard_normal(tuple(out.shape)).astype(np.float32)
    out.backward(torch.from_numpy(gout).to(DEV))

    # ---- fp64 oracle of the same forward / backward ----
    P = {n: p.detach().double().cpu().numpy() for n, p in model.named_parameters()}
    nid = n_id.cpu().numpy()
    nt = node_type.cpu().numpy()[nid]
    loc = local.cpu().numpy()[nid]
    h = np.zeros((nid.size, 32))
    for k, x in x_dict.items():
        m = nt == k
        h[m] = x.double().cpu().numpy()[loc[m]] @ P[f"lins.{k}.weight"].T + P[f"lins.{k}.bias"]
    et = edge_type.cpu().numpy()
    caches = []
    x = h
    ntype = nt
    for i, (ei, e_id, size) in enumerate(adjs):
        ntype = ntype[:size[1]]
        pc = {k[len(f"convs.{i}."):]: v for k, v in P.items() if k.startswith(f"convs.{i}.")}
        o = O.MagREGCNConvOracle(size[1], 7, 10.0, residual=False, use_norm="ln")
        y = o.forward(x, ei[0].cpu().numpy(), ei[1].cpu().numpy(), et[e_id.cpu().numpy()],
                      ntype, pc)
        caches.append((o, y))
        x = np.maximum(y, 0)
    lin = O.Linear(P["out_lin.weight"], P["out_lin.bias"])
    z = lin.forward(x)
    zmax = z.max(1, keepdims=True)
    lse = zmax + np.log(np.exp(z - zmax).sum(1, keepdims=True))
    ref = z - lse
    ok, err = G.close(out.detach().cpu().numpy(), ref, 1e-5)
    assert ok, f"forward rel err {err:.3e}"
    g = gout.astype(np.float64)
    gz = g - np.exp(ref) * g.sum(1, keepdims=True)             # log_softmax VJP
    gx, gr = lin.backward(gz)
    want = {"out_lin.weight": gr["weight"], "out_lin.bias": gr["bias"]}
    for i in range(len(caches) - 1, -1, -1):
        o, y = caches[i]
        gx = gx * (y > 0)
        gx, grc = o.backward(gx)
        for k, v in grc.items():
            want[f"convs.{i}.{k}"] = v
    for name, v in want.items():
        got = dict(model.named_parameters())[name].grad.cpu().numpy()
        ok, err = G.close(got, v, 1e-5)
        assert ok, f"{name}: rel err {err:.3e}"


def test_ns_training_step_reduces_loss():
    from regnn_hip import mag
    from regnn_hip.sampler import NeighborSampler
    gd, rg, edge_type, node_type, local, x_dict, model = _setup(scale=0.005, seed=1)
    n_paper = gd["counts"]["paper"]
    y = torch.full((gd["N"], 1), -1, dtype=torch.int64, device=DEV)
    y[:n_paper, 0] = (torch.arange(n_paper, device=DEV) * 7) % 5     # learnable labels
    smp = NeighborSampler(rg, torch.arange(n_paper, device=DEV), [10, 10], batch_size=256,
                          shuffle=True, seed=5)
    opt = torch.optim.Adam(model.parameters(), lr=1e-2)
    model.train()
    losses = []
    for epoch in range(3):
        smp.set_epoch(epoch)
        for batch in smp:
            losses.append(float(mag.train_step(model, opt, batch, x_dict, edge_type, node_type,
                                               local, y, 1)))
    assert all(np.isfinite(losses))
    assert np.mean(losses[-3:]) < np.mean(losses[:3])


def test_ns_feats_type2_embeddings():
    """feats_type 2 (mag/regnn_ns.py:240-245,306-315): learned embeddings for the non-target
    types + one shared Linear. group_input equals the spec's composition; the tables' gradients
    live only on the rows the batch read (what sparse_rows_allreduce exchanges); loss falls."""
    from regnn_hip import mag, synth
    from regnn_hip.graph import RelGraph
    from regnn_hip.sampler import NeighborSampler
    gd = synth.mag_like(0.003, seed=2, device=DEV)
    keep = gd["rel"] <= 7
    rg = RelGraph(gd["src"][keep], gd["dst"][keep], gd["N"], DEV)
    edge_type = gd["rel"][keep].to(torch.int64) - 1
    node_type = gd["ntype"]
    offs = torch.tensor([gd["type_offsets"][t] for t in synth.NTYPES], device=DEV)
    local = torch.arange(gd["N"], device=DEV) - offs[node_type]
    n_paper = gd["counts"]["paper"]
    x_dict = {0: torch.randn(n_paper, 16, device=DEV)}
    nodes = {k: gd["counts"][t] for k, t in enumerate(synth.NTYPES)}
    torch.manual_seed(0)
    net = mag.REGNN(16, 32, 5, 2, 10.0, 0.0, {k: 16 for k in range(4)}, 7, use_norm="ln",
                    self_loop_type=2, feats_type=2, num_nodes_dict=nodes,
                    target_node_type=0).to(DEV)
    assert set(net.emb_dict.keys()) == {"1", "2", "3"} and not hasattr(net, "lins")
    smp = NeighborSampler(rg, torch.arange(n_paper, device=DEV), [8, 6], batch_size=128,
                          shuffle=True, seed=1)
    bs, n_id, adjs = next(iter(smp))
    h = net.group_input(x_dict, node_type, local, n_id)
    nt, loc = node_type[n_id].cpu(), local[n_id].cpu()
    t = torch.zeros(n_id.numel(), 16, dtype=torch.float64)
    t[nt == 0] = x_dict[0].cpu().double()[loc[nt == 0]]
    for k in (1, 2, 3):
        t[nt == k] = net.emb_dict[str(k)].detach().cpu().double()[loc[nt == k]]
    ref = t @ net.lin.weight.detach().cpu().double().T + net.lin.bias.detach().cpu().double()
    assert torch.allclose(h.detach().cpu().double(), ref, rtol=1e-5, atol=1e-5)
    y = torch.full((gd["N"], 1), -1, dtype=torch.int64, device=DEV)
    y[:n_paper, 0] = (torch.arange(n_paper, device=DEV) * 3) % 5
    opt = torch.optim.Adam(net.parameters(), lr=1e-2)
    net.train()
    mag.train_step(net, opt, (bs, n_id, adjs), x_dict, edge_type, node_type, local, y, 1)
    for p, rows in net.embedding_tables():
        nz = torch.nonzero(p.grad.abs().sum(1)).flatten()
        assert set(nz.tolist()) <= set(rows.tolist())
    losses = []
    for epoch in range(3):
        smp.set_epoch(epoch)
        for batch in smp:
            losses.append(float(mag.train_step(net, opt, batch, x_dict, edge_type, node_type,
                                               local, y, 1)))
    assert np.mean(losses[-3:]) < np.mean(losses[:3])
