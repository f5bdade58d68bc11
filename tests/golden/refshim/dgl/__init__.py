"""TEST-ONLY pure-torch stand-in for the DGL 0.7.1 primitives the reference layer source calls.

It exists so that ``tests/golden/make_golden.py`` can import the reference's own ``layer/`` and
``model/`` files from ``/root/reference`` in THIS container and record golden vectors. It is an
independent restatement of DGL's documented semantics (gather-multiply + ``index_add`` by
destination, per-destination max-subtracted softmax); it is not the product's graph front
(``re-gnn_amd/dgl``) and is never imported by the product, the GPU tests or the bench.
"""
from . import function, base, utils, nn, data  # noqa: F401
from .graph import DGLGraph, remove_self_loop, add_self_loop, graph  # noqa: F401
