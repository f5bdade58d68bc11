"""DGL-compatible graph front over the MI355X kernels (drop-in for the surface RE-GNN uses).

``run_regnn.py`` builds ``dgl.DGLGraph(adjM)``, calls ``remove_self_loop`` / ``add_self_loop`` /
``.to(device)`` / ``.edges()`` (run_regnn.py:84-99), and the layers call ``local_var`` /
``local_scope``, ``ndata`` / ``edata``, ``update_all`` and ``apply_edges``. Message passing on a
ROCm device dispatches to libregnn_hip (regnn_hip.ops); there is no CPU execution path.
"""
from . import function, base, utils, nn, data  # noqa: F401
from .graph import DGLGraph, graph, remove_self_loop, add_self_loop  # noqa: F401
from .base import DGLError  # noqa: F401

__version__ = "0.7.1-regnn-hip"
