"""Drop-in check in THIS container (skipped where /root/reference is absent, e.g. the GPU box):
the reference's own model/REGCN.py, model/REGAT.py and model/REMixHop.py import and construct on
this build's ``layer`` + ``dgl`` packages and produce the same parameter layout as the build's
nets. (Forward needs a ROCm device; parity of forward/backward is covered by the GPU tests on
golden vectors generated from these same reference files.)"""
import importlib
import os
import sys

import pytest
import torch.nn.functional as F

REF = "/root/reference"
pytestmark = pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "model")),
                                reason="reference checkout not present")


def _import_ref_models():
    saved = dict(sys.modules)
    for k in list(sys.modules):
        if k == "model" or k.startswith("model."):
            del sys.modules[k]
    sys.path.insert(1, REF)        # after re-gnn_amd (conftest puts it first): our layer/dgl win
    try:
        import layer
        assert "re-gnn_amd" in layer.__file__
        return (importlib.import_module("model.REGCN").REGCN,
                importlib.import_module("model.REGAT").REGAT,
                importlib.import_module("model.REMixHop").REMixHop)
    finally:
        sys.path.remove(REF)
        for k in list(sys.modules):
            if (k == "model" or k.startswith("model.")) and k not in saved:
                del sys.modules[k]


def _layout(m):
    return {n: tuple(p.shape) for n, p in m.named_parameters()}


def test_reference_models_construct_on_build():
    import dgl
    from regnn_hip import nets
    RREGCN, RREGAT, RREMixHop = _import_ref_models()
    g = dgl.DGLGraph(([0, 1], [1, 0]), num_nodes=2)
    dims = [12, 7]
    a = RREGCN(g, 10, 100.0, 64, 64, 4, 3, F.elu, 0.5, dims)
    b = nets.REGCN(g, 10, 100.0, 64, 64, 4, 3, F.elu, 0.5, dims)
    assert _layout(a) == _layout(b)
    a = RREGAT(g, 10, 100.0, 2, 32, 32, 4, [8, 8, 1], F.elu, 0.5, 0.5, 0.01, False, dims)
    b = nets.REGAT(g, 10, 100.0, 2, 32, 32, 4, [8, 8, 1], F.elu, 0.5, 0.5, 0.01, False, dims)
    assert _layout(a) == _layout(b)
    a = RREMixHop(g, 10, 100.0, 64, 64, 4, 2, dims, input_dropout=0.5, activation=F.elu)
    b = nets.REMixHop(g, 10, 100.0, 64, 64, 4, 2, dims, input_dropout=0.5, activation=F.elu)
    assert _layout(a) == _layout(b)
    # the reference model's layers ARE this build's classes
    assert type(a.layers[0]).__module__ == "layer.REMixHopConv"
