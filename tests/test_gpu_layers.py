"""GPU parity of the drop-in layers / models (HIP path) against the golden vectors made from the
REFERENCE source (tests/golden, fp64) and against the pinned CPU oracle.

Tolerance: fp32 kernels vs fp64 reference, max |err| <= 1e-5 * max(1, max |ref|) per tensor
(BASELINE north star: "within 1e-5 fp32")."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import _golden as G

pytestmark = pytest.mark.gpu
TOL = 1e-5
DEV = "cuda"


def _graph(d):
    import dgl
    return dgl.DGLGraph((d["g_src"], d["g_dst"]), num_nodes=int(d["g_N"])).to(DEV)


def _load(module, d):
    P = {k: torch.from_numpy(v.astype(np.float32)) for k, v in G.sub(d, "p_", np.float32).items()}
    names = {n for n, _ in module.named_parameters()}
    assert names == set(P), names ^ set(P)
    with torch.no_grad():
        for n, p in module.named_parameters():
            p.copy_(P[n])
    return module.to(DEV)


def _check(tag, got, want, tol=TOL):
    got = got.detach().float().cpu().numpy() if torch.is_tensor(got) else got
    ok, err = G.close(got, want, tol)
    assert ok, f"{tag}: rel err {err:.3e} > {tol}"


def _run(module, g, feat_np, gout_np, call):
    feat = torch.from_numpy(feat_np).to(DEV).requires_grad_(True)
    out = call(module, g, feat)
    out.backward(torch.from_numpy(gout_np).to(DEV))
    torch.cuda.synchronize()
    return out, feat.grad


def _grads(module):
    return {n: p.grad for n, p in module.named_parameters() if p.grad is not None}


@pytest.mark.parametrize("name", G.names("regraphconv_"))
def test_regraphconv(name):
    from layer import REGraphConv
    d = G.load(name)
    m = d["meta"]
    g = _graph(d)
    mod = _load(REGraphConv(int(d["g_R"]), m["alpha"], m["in_feats"], m["out_feats"],
                            norm=m["norm"], bias=m["bias"], weight=m["weight"],
                            activation=F.elu if m["activation"] else None), d)
    e_feat = torch.from_numpy(d["g_rel"]).to(DEV)
    out, gfeat = _run(mod, g, d["feat"], d["gout"], lambda mo, gg, f: mo(gg, f, e_feat))
    _check("out", out, d["out"])
    _check("grad_feat", gfeat, d["grad_feat"])
    for k, v in G.sub(d, "grad_").items():
        if k != "feat":
            _check(k, _grads(mod)[k], v)


@pytest.mark.parametrize("name", G.names("regatconv_"))
def test_regatconv(name):
    from layer import REGATConv
    d = G.load(name)
    m = d["meta"]
    g = _graph(d)
    mod = _load(REGATConv(int(d["g_R"]), m["alpha"], m["in_feats"], m["out_feats"],
                          m["num_heads"], 0.0, 0.0, m["negative_slope"], m["residual"],
                          F.elu if m["activation"] else None, use_weight=m["use_weight"]), d)
    e_feat = torch.from_numpy(d["g_rel"]).to(DEV) if m["edge_feats"] else None
    out, gfeat = _run(mod, g, d["feat"], d["gout"], lambda mo, gg, f: mo(gg, f, e_feat))
    _check("out", out, d["out"])
    _check("grad_feat", gfeat, d["grad_feat"])
    for k, v in G.sub(d, "grad_").items():
        if k != "feat":
            _check(k, _grads(mod)[k], v)


@pytest.mark.parametrize("name", G.names("remixhopconv_"))
def test_remixhopconv(name):
    from layer import REMixHopConv
    d = G.load(name)
    m = d["meta"]
    g = _graph(d)
    mod = _load(REMixHopConv(int(d["g_R"]), m["alpha"], m["in_feats"], m["out_feats"], p=m["p"],
                             activation=F.elu if m["activation"] else None), d)
    e_feat = torch.from_numpy(d["g_rel"]).to(DEV)
    out, gfeat = _run(mod, g, d["feat"], d["gout"], lambda mo, gg, f: mo(gg, f, e_feat))
    _check("out", out, d["out"])
    _check("grad_feat", gfeat, d["grad_feat"])
    for k, v in G.sub(d, "grad_").items():
        if k != "feat":
            _check(k, _grads(mod)[k], v)


@pytest.mark.parametrize("name", G.names("model_"))
def test_models(name):
    from regnn_hip import nets
    d = G.load(name)
    m = d["meta"]
    g = _graph(d)
    R, a, C, dims = int(d["g_R"]), m["alpha"], m["n_classes"], m["dims"]
    if m["model"] == "REGCN":
        net = nets.REGCN(g, R, a, 64, 64, C, m["num_layers"], F.elu, 0.0, dims)
    elif m["model"] == "REGAT":
        net = nets.REGAT(g, R, a, m["num_layers"], m["hidden"], m["hidden"], C, m["heads"], F.elu,
                         0.0, 0.0, 0.01, False, dims)
    else:
        net = nets.REMixHop(g, R, a, 64, 64, C, m["num_layers"], dims, input_dropout=0.0,
                            activation=F.elu)
    _load(net, d)
    net.eval()
    feats = [torch.from_numpy(d[f"feat{i}"]).to(DEV) for i in range(len(dims))]
    e_feat = torch.from_numpy(d["g_rel"]).to(DEV)
    logits, emb = net(feats, e_feat)
    logits.backward(torch.from_numpy(d["gout"]).to(DEV))
    _check("logits", logits, d["logits"])
    _check("emb", emb, d["emb"])
    grads = _grads(net)
    for k, v in G.sub(d, "grad_").items():
        _check(k, grads[k], v)


def test_determinism_regraphconv():
    """two runs of forward+backward give bitwise-identical outputs and gradients (no atomics)."""
    from layer import REGraphConv
    d = G.load("regraphconv_norm_weight_bias_elu")
    g = _graph(d)
    e_feat = torch.from_numpy(d["g_rel"]).to(DEV)
    res = []
    for _ in range(2):
        mod = _load(REGraphConv(int(d["g_R"]), 100.0, 64, 64, activation=F.elu), d)
        out, gfeat = _run(mod, g, d["feat"], d["gout"], lambda mo, gg, f: mo(gg, f, e_feat))
        res.append([out, gfeat] + [p.grad for p in mod.parameters()])
    for a, b in zip(*res):
        assert torch.equal(a, b)


def _check_all(mod, d, out, gfeat):
    _check("out", out, d["out"])
    _check("grad_feat", gfeat, d["grad_feat"])
    want = {k: v for k, v in G.sub(d, "grad_").items() if k != "feat"}
    got = _grads(mod)
    assert set(got) == set(want), set(got) ^ set(want)
    for k, v in want.items():
        _check(k, got[k], v)


@pytest.mark.parametrize("name", G.names("resageconv_"))
def test_resageconv(name):
    """layer/RESAGEConv.py: deg^-1 pre-norm + root term, HIP degree/SpMM."""
    from layer import RESAGEConv
    d = G.load(name)
    m = d["meta"]
    mod = _load(RESAGEConv(int(d["g_R"]), m["alpha"], m["in_feats"], m["out_feats"],
                           norm=m["norm"], bias=m["bias"], weight=m["weight"],
                           activation=F.elu if m["activation"] else None), d)
    e_feat = torch.from_numpy(d["g_rel"]).to(DEV)
    out, gfeat = _run(mod, _graph(d), d["feat"], d["gout"], lambda mo, gg, f: mo(gg, f, e_feat))
    _check_all(mod, d, out, gfeat)


@pytest.mark.parametrize("name", G.names("reginconv_"))
def test_reginconv(name):
    """layer/REGINConv.py: sum aggregation (whatever aggregator_type says) + deg^-1 post-norm."""
    from layer import REGINConv
    d = G.load(name)
    m = d["meta"]
    lin = torch.nn.Linear(*m["apply_linear"]) if m["apply_linear"] else None
    mod = _load(REGINConv(int(d["g_R"]), m["alpha"], apply_func=lin,
                          aggregator_type=m["aggregator_type"]), d)
    e_feat = torch.from_numpy(d["g_rel"]).to(DEV)
    out, gfeat = _run(mod, _graph(d), d["feat"], d["gout"], lambda mo, gg, f: mo(gg, f, e_feat))
    _check_all(mod, d, out, gfeat)


@pytest.mark.parametrize("name", G.names("regatv2conv_"))
def test_regatv2conv(name):
    """layer/REGATv2Conv.py: attn . LeakyReLU(fs[u] + fd[v]) scores, edge softmax, head SpMM."""
    from layer import REGATv2Conv
    d = G.load(name)
    m = d["meta"]
    mod = _load(REGATv2Conv(int(d["g_R"]), m["alpha"], m["in_feats"], m["out_feats"],
                            m["num_heads"], 0.0, 0.0, m["negative_slope"], m["residual"],
                            F.elu if m["activation"] else None,
                            share_weights=m["share_weights"]), d)
    e_feat = torch.from_numpy(d["g_rel"]).to(DEV) if m["edge_feats"] else None
    out, gfeat = _run(mod, _graph(d), d["feat"], d["gout"], lambda mo, gg, f: mo(gg, f, e_feat))
    _check_all(mod, d, out, gfeat)
