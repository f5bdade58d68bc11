"""Pin the CPU oracle (oracle/regnn_oracle.py) against golden vectors produced by the REFERENCE
source (tests/golden/make_golden.py). CPU only."""
import numpy as np
import pytest

import _golden as G
from oracle import regnn_oracle as O

TOL = 1e-9 * 0 + 2e-6   # fixtures are fp64 results stored as fp32 -> ~1e-7 rounding


def _graph(d):
    return O.Graph(d["g_src"], d["g_dst"], int(d["g_N"]))


def _check(tag, got, want, tol=TOL):
    ok, err = G.close(got, want, tol)
    assert ok, f"{tag}: rel err {err:.3e}"


@pytest.mark.parametrize("name", G.names("regraphconv_"))
def test_regraphconv(name):
    d = G.load(name)
    m = d["meta"]
    g = _graph(d)
    P = G.sub(d, "p_")
    o = O.REGraphConvOracle(**m)
    out = o.forward(g, d["feat"].astype(np.float64), d["g_rel"], P["edge_weight"],
                    P.get("weight"), P.get("bias"))
    _check("out", out, d["out"])
    gf, gr = o.backward(g, d["gout"].astype(np.float64))
    _check("grad_feat", gf, d["grad_feat"])
    for k, v in G.sub(d, "grad_").items():
        if k == "feat":
            continue
        _check(k, gr[k], v)


@pytest.mark.parametrize("name", G.names("regatconv_"))
def test_regatconv(name):
    d = G.load(name)
    m = d["meta"]
    g = _graph(d)
    P = G.sub(d, "p_")
    o = O.REGATConvOracle(**m)
    out = o.forward(g, d["feat"].astype(np.float64), d["g_rel"], P)
    _check("out", out, d["out"])
    gf, gr = o.backward(g, d["gout"].astype(np.float64))
    _check("grad_feat", gf, d["grad_feat"])
    for k, v in G.sub(d, "grad_").items():
        if k == "feat":
            continue
        _check(k, gr[k], v)


@pytest.mark.parametrize("name", G.names("remixhopconv_"))
def test_remixhopconv(name):
    d = G.load(name)
    m = d["meta"]
    g = _graph(d)
    P = G.sub(d, "p_")
    o = O.REMixHopConvOracle(**m)
    out = o.forward(g, d["feat"].astype(np.float64), d["g_rel"], P)
    _check("out", out, d["out"])
    gf, gr = o.backward(g, d["gout"].astype(np.float64))
    _check("grad_feat", gf, d["grad_feat"])
    for k, v in G.sub(d, "grad_").items():
        if k == "feat":
            continue
        _check(k, gr[k], v)


_EXTRA = {"resageconv_": O.RESAGEConvOracle, "reginconv_": O.REGINConvOracle,
          "regatv2conv_": O.REGATv2ConvOracle}


@pytest.mark.parametrize("name", [n for p in _EXTRA for n in G.names(p)])
def test_other_re_layers(name):
    """RESAGEConv / REGINConv / REGATv2Conv."""
    d = G.load(name)
    cls = next(c for p, c in _EXTRA.items() if name.startswith(p))
    g = _graph(d)
    P = G.sub(d, "p_")
    o = cls(**d["meta"])
    out = o.forward(g, d["feat"].astype(np.float64), d["g_rel"], P)
    _check("out", out, d["out"])
    gf, gr = o.backward(g, d["gout"].astype(np.float64))
    _check("grad_feat", gf, d["grad_feat"])
    want = {k: v for k, v in G.sub(d, "grad_").items() if k != "feat"}
    assert set(want) == set(gr), set(want) ^ set(gr)
    for k, v in want.items():
        _check(k, gr[k], v)


@pytest.mark.parametrize("name", G.names("mag_regcnconv_"))
def test_mag_regcnconv(name):
    d = G.load(name)
    m = d["meta"]
    P = G.sub(d, "p_")
    o = O.MagREGCNConvOracle(**m)
    out = o.forward(d["x"].astype(np.float64), d["src"], d["dst"], d["edge_type"],
                    d["target_node_type"], P)
    _check("out", out, d["out"])
    gx, gr = o.backward(d["gout"].astype(np.float64))
    _check("grad_x", gx, d["grad_x"])
    for k, v in G.sub(d, "grad_").items():
        if k == "x":
            continue
        _check(k, gr[k], v)


def _feats(d):
    return [d[f"feat{i}"].astype(np.float64) for i in range(len(d["meta"]["dims"]))]


@pytest.mark.parametrize("name", G.names("model_"))
def test_models(name):
    d = G.load(name)
    m = d["meta"]
    g = _graph(d)
    P = G.sub(d, "p_")
    gout = d["gout"].astype(np.float64)
    if m["model"] == "REGCN":
        logits, emb, grads = O.regcn_model(g, _feats(d), d["g_rel"], P, m["num_layers"],
                                           m["alpha"], gout)
    elif m["model"] == "REGAT":
        logits, emb, grads = O.regat_model(g, _feats(d), d["g_rel"], P, m["num_layers"],
                                           m["heads"], m["hidden"], m["alpha"], gout)
    else:
        logits, emb, grads = O.remixhop_model(g, _feats(d), d["g_rel"], P, m["num_layers"],
                                              m["hidden"], m["alpha"], gout)
    _check("logits", logits, d["logits"])
    _check("emb", emb, d["emb"])
    want = G.sub(d, "grad_")
    assert set(want) == set(grads), set(want) ^ set(grads)
    for k, v in want.items():
        _check(k, grads[k], v)


@pytest.mark.parametrize("keep16,ev", [(32768, 4), (16384, 8), (int(0.7 * 65536), 4),
                                       (int(0.9 * 65536), 8)])
def test_dropout_mask_spec(keep16, ev):
    """the fused-dropout mask restatement (include/regnn_hip.h regnn_spmm_fwd_dropout): keep rate,
    no correlation between neighbouring features / rows, a different mask per seed."""
    m = O.dropout_mask(0xDEADBEEF12345, 4000, 16 * ev, ev, keep16)
    keep = keep16 / 65536
    assert abs(m.mean() - keep) < 0.005
    c = m - m.mean()
    assert abs((c[:, 1:] * c[:, :-1]).mean()) < 0.01 * keep
    assert abs((c[1:] * c[:-1]).mean()) < 0.01 * keep
    m2 = O.dropout_mask(0xDEADBEEF12346, 4000, 16 * ev, ev, keep16)
    assert abs((m == m2).mean() - (keep ** 2 + (1 - keep) ** 2)) < 0.01


@pytest.mark.parametrize("name", G.names("mag_regatconv_") + G.names("mag_regatv2conv_"))
def test_mag_regatconv(name):
    """mag REGATConv / REGATv2Conv with the global-max edge softmax."""
    d = G.load(name)
    m = d["meta"]
    P = G.sub(d, "p_")
    o = O.MagREGATConvOracle(v2="v2" in m["layer"], **m)
    out = o.forward(d["x"].astype(np.float64), d["src"], d["dst"], d["edge_type"],
                    d["target_node_type"], P)
    _check("out", out, d["out"])
    gx, gr = o.backward(d["gout"].astype(np.float64))
    _check("grad_x", gx, d["grad_x"])
    want = {k: v for k, v in G.sub(d, "grad_").items() if k != "x"}
    assert set(want) == set(gr), set(want) ^ set(gr)
    for k, v in want.items():
        _check(k, gr[k], v)


def _regnn_adjs(d):
    return [(d[f"adj{h}_src"], d[f"adj{h}_dst"], d[f"adj{h}_eid"], tuple(int(v) for v in d[f"adj{h}_size"]))
            for h in range(d["meta"]["num_layers"])]


@pytest.mark.parametrize("name", [n for n in G.names("mag_regnn_") if n != "mag_regnn_init"])
def test_mag_regnn_model(name):
    """the oracle's REGNN composition (group_input, 2 x REGCNConv + relu, out_lin, log_softmax,
    nll) against the reference's own REGNN class run on a sampled batch (make_golden.gen_regnn)."""
    d = G.load(name)
    m = d["meta"]
    P = G.sub(d, "p_")
    x_dict = {t: d[f"x{t}"].astype(np.float64) for t in range(4) if f"x{t}" in d}
    logp, loss, gr = O.mag_regnn_model(x_dict, d["ntype"], d["local"], d["n_id"], _regnn_adjs(d),
                                       d["edge_type"], P, d["y"][d["batch"]],
                                       feats_type=m["feats_type"],
                                       residual=m.get("residual", False))
    _check("logp", logp, d["logp"])
    _check("loss", np.asarray(loss), d["loss"])
    want = G.sub(d, "grad_")
    assert set(want) == set(gr), set(want) ^ set(gr)
    for k, v in want.items():
        _check(k, gr[k], v)
