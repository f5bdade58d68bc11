"""BASELINE configs 1-4 at their own shapes against the fp64 oracle (VERDICT r1 "next" 1a/1b).

* configs 1/2 — DBLP REGCN 2-layer hidden 64: the synthetic DBLP-shape graph (N = 26,128,
  E = 265,694 with self loops, R = 10) is written in the preprocessed layout
  utils/data.py reads, read back through ``data.load_data`` and turned into the graph and relation
  ids the way run_regnn.py:84-99 does (``data.build_graph``); then the model/REGCN.py wiring
  (``nets.REGCN``) runs forward + backward in eval mode. fp32 against
  ``oracle.regcn_model`` at 1e-5; bf16 feature storage (configs[1]'s dtype, fp32 accumulation)
  against the same fp64 oracle at 1e-2.
* config 3 — ACM REGAT 2 layers, hidden 64, heads [8, 8, 1] (the last layer applied twice,
  model/REGAT.py:61-64), negative slope 0.01, against ``oracle.regat_model``.
* config 4 — IMDB REMixHop p = [0, 1, 2], hidden 64, 2 layers, against ``oracle.remixhop_model``.

Parameters: the models' own seeded init, relation tables drawn so that alpha * w ~ U(-0.5, 1.5)
(both LeakyReLU slopes, weighted degrees below 1: the clamp), biases N(0, 0.1).
Tolerance: max |err| <= tol * max(1, max |ref|) per tensor (tests/_golden.close).
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import _golden as G
from oracle import regnn_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"
ALPHA = 100.0


def _check(tag, got, want, tol):
    got = got.detach().double().cpu().numpy() if torch.is_tensor(got) else got
    ok, err = G.close(got, want, tol)
    assert ok, f"{tag}: rel err {err:.3e} > {tol}"


def _roundtrip(tmp_path, dataset, gd, n_etype, feats):
    """synthetic graph -> preprocessed files -> load_data -> build_graph (run_regnn.py:84-99)."""
    from regnn_hip import data
    src, dst, rel = (gd[k].cpu().numpy() for k in ("src", "dst", "rel"))
    adjM, adjMM, wsl, wsl2 = data.matrices_from_edges(src, dst, rel, gd["N"], n_etype)
    ntype = gd["ntype"].cpu().numpy()
    labels = np.zeros(int((ntype == 0).sum()), np.int64)
    tvt = {"train_idx": np.arange(8), "val_idx": np.arange(8, 10), "test_idx": np.arange(10, 12)}
    prefix = str(tmp_path / dataset)
    data.save_preprocessed(prefix, dataset, [f.cpu().numpy() for f in feats], adjM, adjMM, wsl,
                           wsl2, ntype, labels, tvt)
    _, feats_l, adjM2, _, _, wsl2_2, _, _, _ = data.load_data(dataset, prefix)
    g, e_feat = data.build_graph(adjM2, wsl2_2, device=DEV)
    s, d = g.edges()
    og = O.Graph(s.cpu().numpy(), d.cpu().numpy(), gd["N"])
    rel_np = e_feat.cpu().numpy()
    assert rel_np.min() >= 1 and rel_np.max() <= gd["R"]
    return g, e_feat, og, rel_np, feats_l


def _set_params(net, seed):
    gen = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for n, p in net.named_parameters():
            if n.endswith("edge_weight"):
                p.copy_((torch.rand(p.shape, generator=gen) * 2.0 - 0.5) / ALPHA)
            elif n.endswith("bias"):
                p.copy_(torch.randn(p.shape, generator=gen) * 0.1)
    return {n: p.detach().double().cpu().numpy() for n, p in net.named_parameters()}


def _grads(net):
    return {n: p.grad for n, p in net.named_parameters() if p.grad is not None}


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_dblp_regcn2_vs_oracle(tmp_path, dtype):
    """configs 1/2: DBLP REGCN-2 hidden 64 through the run_regnn.py graph plumbing."""
    from regnn_hip import nets, synth
    gd = synth.dblp_like(seed=0, device="cpu")
    feats = synth.type_features(gd["counts"], synth.DBLP_DIMS, seed=1, device="cpu", kind="dblp")
    g, e_feat, og, rel, feats_l = _roundtrip(tmp_path, "DBLP", gd, 6, feats)
    assert 0.99 * 265_694 < og.E <= 265_694        # duplicate (u, v) pairs collapse
    dims = [f.shape[1] for f in feats_l]
    torch.manual_seed(0)
    net = nets.REGCN(g, gd["R"], ALPHA, 64, 64, 4, 2, F.elu, 0.5, dims)
    P = _set_params(net, 1)
    net = net.to(DEV).eval()
    tdt = torch.float32 if dtype == "fp32" else torch.bfloat16
    x = [torch.from_numpy(f).to(DEV, tdt) for f in feats_l]
    gout = np.random.default_rng(2).standard_normal((gd["N"], 4)).astype(np.float32)
    emb = net.embed(x, e_feat)
    logits = F.linear(emb.float(), net.out_lin.weight, net.out_lin.bias)
    logits.backward(torch.from_numpy(gout).to(DEV))
    torch.cuda.synchronize()
    f64 = [f.astype(np.float64) for f in feats_l]
    want_logits, want_emb, want_g = O.regcn_model(og, f64, rel, P, 2, ALPHA,
                                                  gout.astype(np.float64))
    tol = 1e-5 if dtype == "fp32" else 1e-2
    _check("logits", logits, want_logits, tol)
    _check("emb", emb, want_emb, tol)
    got = _grads(net)
    assert set(got) == set(want_g), set(got) ^ set(want_g)
    for k, v in want_g.items():
        _check(k, got[k], v, tol)


def test_acm_regat_h8_vs_oracle(tmp_path):
    """config 3: ACM REGAT 2 layers, hidden 64, heads [8, 8, 1] (last layer twice)."""
    from regnn_hip import nets, synth
    gd = synth.acm_like(seed=0, device="cpu")
    feats = synth.type_features(gd["counts"], synth.ACM_DIMS, seed=1, device="cpu", kind="target")
    g, e_feat, og, rel, feats_l = _roundtrip(tmp_path, "ACM", gd, 4, feats)
    # kind="target" leaves the non-target types all-zero: give them signal so every input
    # Linear's gradient is non-trivial
    rng = np.random.default_rng(5)
    feats_l = [f if i == 0 else rng.standard_normal(f.shape).astype(np.float32)
               for i, f in enumerate(feats_l)]
    dims = [f.shape[1] for f in feats_l]
    torch.manual_seed(0)
    net = nets.REGAT(g, gd["R"], ALPHA, 2, 64, 64, 3, [8, 8, 1], F.elu, 0.0, 0.0, 0.01, False,
                     dims)
    P = _set_params(net, 3)
    net = net.to(DEV).eval()
    x = [torch.from_numpy(f).to(DEV) for f in feats_l]
    gout = np.random.default_rng(4).standard_normal((gd["N"], 3)).astype(np.float32)
    logits, emb = net(x, e_feat)
    logits.backward(torch.from_numpy(gout).to(DEV))
    torch.cuda.synchronize()
    want_logits, want_emb, want_g = O.regat_model(og, [f.astype(np.float64) for f in feats_l],
                                                  rel, P, 2, [8, 8, 1], 64, ALPHA,
                                                  gout.astype(np.float64), slope=0.01)
    _check("logits", logits, want_logits, 1e-5)
    _check("emb", emb, want_emb, 1e-5)
    got = _grads(net)
    for k, v in want_g.items():
        _check(k, got[k], v, 1e-5)


def test_imdb_remixhop_vs_oracle(tmp_path):
    """config 4: IMDB REMixHop p = [0, 1, 2], hidden 64, 2 layers, ELU."""
    from regnn_hip import nets, synth
    gd = synth.imdb_like(seed=0, device="cpu")
    feats = synth.type_features(gd["counts"], synth.IMDB_DIMS, seed=1, device="cpu",
                                kind="target")
    g, e_feat, og, rel, feats_l = _roundtrip(tmp_path, "IMDB", gd, 4, feats)
    rng = np.random.default_rng(6)
    feats_l = [f if i == 0 else rng.standard_normal(f.shape).astype(np.float32)
               for i, f in enumerate(feats_l)]
    dims = [f.shape[1] for f in feats_l]
    torch.manual_seed(0)
    net = nets.REMixHop(g, gd["R"], ALPHA, 64, 64, 3, 2, dims, input_dropout=0.0,
                        activation=F.elu)
    P = _set_params(net, 7)
    net = net.to(DEV).eval()
    x = [torch.from_numpy(f).to(DEV) for f in feats_l]
    gout = np.random.default_rng(8).standard_normal((gd["N"], 3)).astype(np.float32)
    logits, emb = net(x, e_feat)
    logits.backward(torch.from_numpy(gout).to(DEV))
    torch.cuda.synchronize()
    want_logits, want_emb, want_g = O.remixhop_model(og, [f.astype(np.float64) for f in feats_l],
                                                     rel, P, 2, 64, ALPHA,
                                                     gout.astype(np.float64))
    _check("logits", logits, want_logits, 1e-5)
    _check("emb", emb, want_emb, 1e-5)
    got = _grads(net)
    for k, v in want_g.items():
        _check(k, got[k], v, 1e-5)


def test_reference_edge_loop_on_device_graph():
    """run_regnn.py:84-99 as written: g.to(device), then e_feat from a Python loop over
    zip(*g.edges()) with u.cpu().item(). The ends are device tensors (DGL semantics) whose
    iteration reads one host copy, and the relation ids equal the vectorised build's."""
    import time
    import dgl
    from regnn_hip import data, synth
    gd = synth.acm_like(seed=1, device="cpu")
    adjM, _, _, wsl2 = data.matrices_from_edges(gd["src"].numpy(), gd["dst"].numpy(),
                                                gd["rel"].numpy(), gd["N"], int(gd["R"]) - 3)
    g = dgl.add_self_loop(dgl.remove_self_loop(dgl.DGLGraph(adjM))).to(DEV)
    s, d = g.edges()
    assert s.is_cuda and d.is_cuda and type(s * 1) is torch.Tensor
    t0 = time.perf_counter()
    e_feat = []
    for u, v in zip(*g.edges()):
        e_feat.append(wsl2[(u.cpu().item(), v.cpu().item())])
    dt = time.perf_counter() - t0
    _, e_vec = data.build_graph(adjM, wsl2, device=DEV)
    assert torch.equal(torch.tensor(e_feat, dtype=torch.long), e_vec.cpu())
    print(f"{len(e_feat)} edges in {dt:.2f} s")
