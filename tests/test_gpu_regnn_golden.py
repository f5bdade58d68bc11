"""The neighbour-sampled REGNN (mag/regnn_ns.py:216-346) + nll_loss (:404) against golden vectors
made by running the REFERENCE's own REGNN class on a sampled batch (tests/golden/make_golden.py
gen_regnn, fp64): the autograd path (mag.REGNN, feats_type 3 and 2) and the fused step
(regnn_nsm_step over the device sampler's blocks, feats_type 3). Sampled neighbourhoods come
from the build's sampler spec; the device sampler reproduces the fixture's n_id bit for bit.
Tolerance 1e-5 x max(1, max|ref|) per tensor."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import _golden as G

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL = 1e-5


def _check(tag, got, want, tol=TOL):
    got = got.detach().double().cpu().numpy() if torch.is_tensor(got) else np.asarray(got)
    ok, err = G.close(got, want, tol)
    assert ok, f"{tag}: rel err {err:.3e}"


def _model(d):
    from regnn_hip import mag
    m = d["meta"]
    counts = m["counts"]
    K = m["in_channels"]
    dims = m.get("feature_dims", [K] * 4)          # feats_type 5: paper rows 256-d, others 128
    model = mag.REGNN(K, m["hidden"], m["classes"], m["num_layers"], m["scaling_factor"], 0.0,
                      {t: dims[t] for t in range(4)}, m["num_edge_types"],
                      residual=m.get("residual", False), use_norm="ln",
                      self_loop_type=2, feats_type=m["feats_type"],
                      num_nodes_dict={t: counts[t] for t in range(4)}, target_node_type=0)
    P = G.sub(d, "p_", np.float32)
    assert {n for n, _ in model.named_parameters()} == set(P)
    with torch.no_grad():
        for n, p in model.named_parameters():
            p.copy_(torch.from_numpy(P[n]))
    return model.to(DEV)


def _inputs(d):
    x_dict = {t: torch.from_numpy(d[f"x{t}"]).to(DEV) for t in range(4) if f"x{t}" in d}
    adjs = [(torch.from_numpy(np.stack([d[f"adj{h}_src"], d[f"adj{h}_dst"]])).to(DEV),
             torch.from_numpy(d[f"adj{h}_eid"]).to(DEV),
             tuple(int(v) for v in d[f"adj{h}_size"])) for h in range(d["meta"]["num_layers"])]
    return (x_dict, adjs, torch.from_numpy(d["edge_type"]).to(DEV),
            torch.from_numpy(d["ntype"]).to(DEV), torch.from_numpy(d["local"]).to(DEV))


# (mag_regnn_init holds seeded initial parameters only: tests/test_cpu_mag_init.py)
REGNN_CASES = [n for n in G.names("mag_regnn_") if n != "mag_regnn_init"]


@pytest.mark.parametrize("name", REGNN_CASES)
def test_regnn_autograd_path_vs_reference(name):
    d = G.load(name)
    model = _model(d)
    model.eval()
    x_dict, adjs, et, nt, loc = _inputs(d)
    n_id = torch.from_numpy(d["n_id"]).to(DEV)
    out = model(n_id, x_dict, adjs, et, nt, loc)
    loss = F.nll_loss(out, torch.from_numpy(d["y"][d["batch"]]).to(DEV))
    loss.backward()
    _check("logp", out, d["logp"])
    _check("loss", loss, d["loss"])
    got = {n: p.grad for n, p in model.named_parameters()}
    for k, v in G.sub(d, "grad_").items():
        _check(k, got[k], v)


@pytest.mark.parametrize("name,lean", [("mag_regnn_ft3", "off"), ("mag_regnn_schema", "on"),
                                       ("mag_regnn_schema", "off")])
def test_regnn_fused_step_vs_reference(monkeypatch, name, lean):
    """regnn_ns_hop reproduces the fixture's sampled batch; regnn_nsm_step's loss and every
    gradient match the reference REGNN's.
    * mag_regnn_ft3: relations drawn at random (not one per (target type, source type) pair),
      so layer 0 takes the edge pass (rel_slots 0); the full last hop, whose outermost n_id and
      per-edge local ids are checked against the fixture;
    * mag_regnn_schema: the ogbn-mag schema (make_golden._mag_schema_graph), K = 128, hidden
      64, 349 classes, fan-out [25, 20] -- the mode bench.py times: relation slots on and the
      meta-only last hop (n_id checked up to the layer-0 targets), and the full hop."""
    from regnn_hip import ns
    from regnn_hip.graph import RelGraph
    from regnn_hip.ns import DeviceSampler, FusedStep
    monkeypatch.setitem(ns.LEAN_LAST_HOP, "mode", lean)
    d = G.load(name)
    m = d["meta"]
    N = int(sum(m["counts"]))
    rg = RelGraph(torch.from_numpy(d["src"]), torch.from_numpy(d["dst"]), N, DEV)
    ds = DeviceSampler(rg, m["sizes"], len(d["batch"]), etype=torch.from_numpy(d["edge_type"]),
                       ntype=torch.from_numpy(d["ntype"]), num_edge_types=m["num_edge_types"])
    model = _model(d)
    model.eval()
    for p in model.parameters():
        p.grad = torch.zeros_like(p)
    x_dict, _, _, nt, loc = _inputs(d)
    if m.get("y_global"):
        y_flat = torch.from_numpy(d["y"])
    else:
        y_flat = torch.full((N,), -1, dtype=torch.int64)
        y_flat[:m["counts"][0]] = torch.from_numpy(d["y"])
    loss = torch.zeros((), device=DEV)
    fs = FusedStep(model, ds, x_dict, nt, loc, y_flat, loss)
    assert fs.P.rel_slots == (1 if m.get("schema") == "ogbn-mag" else 0)
    L_ = len(m["sizes"])
    assert ds.meta_only[L_ - 1] == (lean == "on")
    with pytest.raises(RuntimeError):                  # the hops have not run since
        fs.step()
    ds.set_seed(m["seed"], m["epoch"], m["batch_idx"])
    ds.set_targets(torch.from_numpy(d["batch"]).to(DEV))
    ds.run_hops()
    # the sampled blocks' sizes: hop h's (n_src, n_dst) of the fixture (adjs outermost first)
    for h in range(L_):
        n_src, n_dst = (int(v) for v in d[f"adj{L_ - 1 - h}_size"])
        assert int(ds.sizes[h]) == n_dst
        E_h = int(ds.sizes[8 + h])
        assert E_h == d[f"adj{L_ - 1 - h}_src"].size + n_dst          # + one self loop per row
    n_chk = int(ds.sizes[L_ if lean == "off" else L_ - 1])
    assert ds.n_id[:n_chk].cpu().numpy().tolist() == d["n_id"][:n_chk].tolist()
    if lean == "off":
        assert n_chk == d["n_id"].size
        # the sampler's per-edge source type / table row of the last hop (layer 0's block; in
        # the strided layout, its non-empty slots)
        et, eo = ds.edge_meta[L_ - 1]
        blk = ds.blocks[L_ - 1]
        if ds.strided:
            ix = blk.csr_idx.long()
            keep = ix >= 0
        else:
            E = int(ds.sizes[8 + L_ - 1])
            ix = blk.csr_idx[:E].long()
            keep = torch.ones_like(ix, dtype=torch.bool)
        g = ds.n_id.long()[ix[keep]]
        assert torch.equal(et[:ix.numel()][keep].long(), nt.to(DEV).long()[g])
        assert torch.equal(eo[:ix.numel()][keep], loc.to(DEV).long()[g])
    fs.step()
    torch.cuda.synchronize()
    _check("loss", loss, d["loss"])
    got = {n: p.grad for n, p in model.named_parameters()}
    for k, v in G.sub(d, "grad_").items():
        _check(k, got[k], v)


@pytest.mark.parametrize("lean", ["on", "off"])
def test_regnn_module_step_ft5_vs_reference(monkeypatch, lean):
    """the reference's default NS model shape outside the fused step --
    feats_type 5's unequal input widths (paper 256-d, others 128-d), hidden 128, residual --
    through NSTrainer's module path on the device sampler (typed first layer with the meta-only
    last hop, or the full hop), against the reference REGNN's loss and every gradient (1e-5)."""
    from regnn_hip import ns
    from regnn_hip.graph import RelGraph
    from regnn_hip.ns import NSTrainer
    monkeypatch.setitem(ns.MODULE_LEAN_HOP, "mode", lean)
    d = G.load("mag_regnn_ft5_h128")
    m = d["meta"]
    N = int(sum(m["counts"]))
    rg = RelGraph(torch.from_numpy(d["src"]), torch.from_numpy(d["dst"]), N, DEV)
    model = _model(d)
    model.eval()
    x_dict, _, et, nt, loc = _inputs(d)
    y = torch.from_numpy(d["y"]).to(DEV).reshape(-1, 1)
    batch = torch.from_numpy(d["batch"]).to(DEV)
    tr = NSTrainer(model, None, rg, m["sizes"], batch.numel(), batch, x_dict, et, nt, loc, y,
                   m["num_edge_types"], seed=m["seed"], engine="auto", pipeline=False)
    assert tr.fused is None                     # hidden 128 / residual: the module path
    s = tr.slots[0]
    s.set_seed(m["seed"], m["epoch"], m["batch_idx"])
    s.set_targets(batch)
    s.run_hops(meta_only=tr._module_lean, strided=False)
    L_ = len(m["sizes"])
    n_chk = int(s.sizes[L_ - 1 if tr._module_lean else L_])
    assert s.n_id[:n_chk].cpu().numpy().tolist() == d["n_id"][:n_chk].tolist()
    tr._module_step(s)
    torch.cuda.synchronize()
    _check("loss", tr.loss, d["loss"])
    got = {n: p.grad for n, p in model.named_parameters()}
    for k, v in G.sub(d, "grad_").items():
        _check(k, got[k], v)
