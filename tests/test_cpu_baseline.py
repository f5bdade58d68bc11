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
