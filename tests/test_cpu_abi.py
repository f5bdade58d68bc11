"""CPU-side checks of the C-ABI boundary: the library builds/loads and exports exactly the
symbols include/regnn_hip.h declares; wrappers refuse CPU tensors (no CPU fallback)."""
import os
import re
import subprocess

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "regnn_hip.h")


def declared():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|int64_t)\s+(regnn_\w+)\s*\(", src, re.M)))


def test_library_exports_header_symbols():
    from regnn_hip import _lib
    decl = declared()
    assert decl, "no declarations parsed"
    assert sorted(_lib.EXPORTED) == decl
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB], capture_output=True,
                         text=True).stdout
    syms = set(re.findall(r"\bT (regnn_\w+)", out))
    assert set(decl) <= syms, set(decl) - syms


def test_abi_version_and_slab():
    from regnn_hip import _lib
    assert _lib._so.regnn_abi_version() == _lib.ABI_VERSION
    assert _lib.slab_rows() >= 2048


def test_invalid_arguments_rejected_without_gpu():
    """argument validation happens before any launch: NULL ptr array -> EINVAL (1)."""
    from regnn_hip import _lib
    rc = _lib._so.regnn_spmm_fwd(None, None, None, None, None, None, None, None, None, None,
                                 10, 64, 0, 0, 0, None, 0, None, None, 0, None, None, 0, None, None)
    assert rc == 1
    rc = _lib._so.regnn_degree_bwd(None, None, None, None, 5, -0.5, 100, 0, None, 0, None, None,
                                   None)
    assert rc == 1
    # regnn_row_scale: NULL rows, z without dot, keep threshold > 2^16 -> EINVAL; 0 rows -> OK
    rs = _lib._so.regnn_row_scale
    assert rs(None, None, None, 4, 64, 0, None, 0, 1.0, None, None, None) == 1
    assert rs(1 << 20, None, 1 << 21, 4, 64, 0, None, 0, 1.0, 1 << 22, None, None) == 1
    assert rs(1 << 20, None, 1 << 21, 4, 64, 0, 1 << 23, 65537, 2.0, None, None, None) == 1
    assert rs(None, None, None, 0, 64, 0, None, 0, 1.0, None, None, None) == 0


def test_cpu_tensor_refused():
    from regnn_hip import _lib
    with pytest.raises(RuntimeError, match="no CPU path"):
        _lib.ptr(torch.zeros(3))


def test_layer_package_surface():
    import layer
    import dgl
    for name in ("REGraphConv", "REGATConv", "REMixHopConv", "RESAGEConv", "REGATv2Conv",
                 "REGINConv"):
        assert hasattr(layer, name)
    for name in ("DGLGraph", "remove_self_loop", "add_self_loop", "function"):
        assert hasattr(dgl, name)
    from dgl.nn.pytorch.softmax import edge_softmax  # noqa: F401
    from dgl.nn.pytorch.utils import Identity  # noqa: F401
    from dgl.nn.pytorch.conv import GraphConv, GATConv  # noqa: F401
    from dgl.data import CiteseerGraphDataset  # noqa: F401


def test_state_dict_keys_match_reference_layout():
    """parameter names / shapes of the drop-in layers equal the reference's (golden fixtures)."""
    import numpy as np
    import _golden as G
    from layer import REGraphConv, REGATConv, REMixHopConv
    d = G.load("regraphconv_norm_weight_bias_elu")
    m = REGraphConv(int(d["g_R"]), 100.0, 64, 64)
    want = {k: v.shape for k, v in G.sub(d, "p_").items()}
    assert {n: tuple(p.shape) for n, p in m.named_parameters()} == want
    d = G.load("regatconv_h8_d64_ee_res_elu")
    mm = d["meta"]
    m = REGATConv(int(d["g_R"]), 100.0, mm["in_feats"], mm["out_feats"], mm["num_heads"],
                  residual=True)
    assert {n: tuple(p.shape) for n, p in m.named_parameters()} == \
        {k: v.shape for k, v in G.sub(d, "p_").items()}
    d = G.load("remixhopconv_f64")
    m = REMixHopConv(int(d["g_R"]), 100.0, 64, 64)
    assert {n: tuple(p.shape) for n, p in m.named_parameters()} == \
        {k: v.shape for k, v in G.sub(d, "p_").items()}
    assert np.isfinite(d["out"]).all()


def test_dgl_front_structure():
    import numpy as np
    import scipy.sparse as sp
    import dgl
    A = sp.random(30, 30, density=0.2, random_state=0, format="csr")
    A.setdiag(1.0)
    g = dgl.add_self_loop(dgl.remove_self_loop(dgl.DGLGraph(A)))
    s, d = g.edges()
    assert g.number_of_nodes() == 30
    assert (s[-30:] == torch.arange(30)).all() and (d[-30:] == torch.arange(30)).all()
    nnz_off = A.nnz - 30
    assert s.numel() == nnz_off + 30
    coo = A.tocoo()
    keep = coo.row != coo.col
    assert np.array_equal(s[:-30].numpy(), coo.row[keep])
    with pytest.raises(Exception, match="ROCm"):
        g.relgraph("cpu")
