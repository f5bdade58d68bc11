"""The bench's CPU baseline (oracle/cpu_regcn.py: torch.sparse CSR restatement of REGraphConv,
BASELINE.md §3) pinned to the golden vectors of the shim-run reference layer
(layer/REGraphConv.py:52-106, weightless norm=True layer: forward, d feat, d edge_weight)."""
import numpy as np
import torch

import _golden as G
from oracle import cpu_regcn as C


def test_cpu_baseline_layer_matches_golden():
    d = G.load("regraphconv_norm_noweight")
    g = C.CsrGraph(d["g_src"], d["g_dst"], int(d["g_N"]))
    rel = C.rel_csr_of(g, d["g_rel"])
    lay = C.REGraphConvCPU(d["meta"]["alpha"])
    x = torch.from_numpy(d["feat"].astype(np.float64))
    w = torch.from_numpy(d["p_edge_weight"].astype(np.float64))
    out = lay.forward(g, x, rel, w)
    gx, gw = lay.backward(g, torch.from_numpy(d["gout"].astype(np.float64)))
    for got, want, name in ((out, d["out"], "out"), (gx, d["grad_feat"], "grad_feat"),
                            (gw, d["grad_edge_weight"], "grad_edge_weight")):
        ok, err = G.close(got.numpy(), want, 1e-5)
        assert ok, f"{name}: rel err {err:.3e}"


def test_cpu_baseline_fp32_stack_runs():
    """the timed unit (2-layer stack, fp32) on a small synthetic graph: finite, right shapes."""
    rng = np.random.default_rng(0)
    N, E = 500, 6000
    src, dst = rng.integers(0, N, E), rng.integers(0, N, E)
    rel = rng.integers(1, 8, E)
    g = C.CsrGraph(src, dst, N)
    r = C.rel_csr_of(g, rel)
    layers = [C.REGraphConvCPU(100.0) for _ in range(2)]
    ws = [torch.full((7, 1), 0.01) for _ in range(2)]
    h, gx, gws = C.regcn_stack_step(g, layers, torch.randn(N, 64), r, ws)
    assert h.shape == (N, 64) and gx.shape == (N, 64) and len(gws) == 2
    assert torch.isfinite(gx).all() and all(torch.isfinite(v).all() for v in gws)


def test_cpu_ns_sampler_bit_exact():
    """oracle/cpu_ns.Sampler (the numpy-vectorised sampler of the NS CPU baseline) equals
    sampler_oracle.neighbor_sample: n_id, local edge lists, CSR positions, sizes."""
    from oracle import cpu_ns as CN
    from oracle import sampler_oracle as SO
    rng = np.random.default_rng(4)
    N, E = 900, 12000
    dst = np.minimum((rng.pareto(1.1, E) * 3).astype(np.int64), N - 1)
    src = rng.integers(0, N, E)
    o = np.argsort(dst, kind="stable")
    src, dst = src[o], dst[o]
    ptr = np.zeros(N + 1, np.int64)
    ptr[1:] = np.cumsum(np.bincount(dst, minlength=N))
    smp = CN.Sampler(ptr, src, N)
    for bi, batch in enumerate([np.arange(40), rng.permutation(N)[:33], np.array([0, 1, 2])]):
        n_id, adjs = smp.sample(batch, [9, 5], 77, 1, bi)
        _, rn_id, radjs = SO.neighbor_sample(ptr, src, batch.tolist(), [9, 5], 77, 1, bi)
        assert n_id.tolist() == rn_id
        for (s, d, p, sz), (rs, rd, re, rsz) in zip(adjs, radjs):
            assert s.tolist() == rs and d.tolist() == rd and p.tolist() == re
            assert tuple(sz) == tuple(rsz)


def test_cpu_ns_model_matches_reference_regnn():
    """oracle/cpu_ns.REGNNCPU (the NS CPU baseline's model) against the reference REGNN's golden
    vectors on the ogbn-mag-schema batch (make_golden.gen_regnn_schema): log-probabilities, loss
    and every parameter gradient at 1e-5 (fp64)."""
    from oracle import cpu_ns as CN
    d = G.load("mag_regnn_schema")
    m = d["meta"]
    model = CN.REGNNCPU(m["in_channels"], m["hidden"], m["classes"], m["num_layers"],
                        m["scaling_factor"], 0.0, 4).double()
    P = G.sub(d, "p_")
    assert {n for n, _ in model.named_parameters()} == set(P)
    with torch.no_grad():
        for n, p in model.named_parameters():
            p.copy_(torch.from_numpy(P[n]))
    model.eval()
    x_dict = {t: torch.from_numpy(d[f"x{t}"].astype(np.float64)) for t in range(4)}
    adjs = [(torch.from_numpy(d[f"adj{h}_src"]), torch.from_numpy(d[f"adj{h}_dst"]),
             torch.from_numpy(d[f"adj{h}_eid"]), tuple(int(v) for v in d[f"adj{h}_size"]))
            for h in range(m["num_layers"])]
    out = model(torch.from_numpy(d["n_id"]), x_dict, adjs, torch.from_numpy(d["edge_type"]),
                torch.from_numpy(d["ntype"]), torch.from_numpy(d["local"]))
    loss = torch.nn.functional.nll_loss(out, torch.from_numpy(d["y"][d["batch"]]))
    loss.backward()
    for got, want, name in ((out, d["logp"], "logp"), (loss, d["loss"], "loss")):
        ok, err = G.close(got.detach().numpy(), want, 1e-5)
        assert ok, f"{name}: rel err {err:.3e}"
    want = G.sub(d, "grad_")
    for n, p in model.named_parameters():
        if n not in want:
            assert p.grad is None, n                       # REGNN.norm: declared, unused
            continue
        ok, err = G.close(p.grad.numpy(), want[n], 1e-5)
        assert ok, f"{n}: rel err {err:.3e}"
