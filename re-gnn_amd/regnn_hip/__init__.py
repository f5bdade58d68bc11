"""regnn_hip — MI355X-native kernels + host runtime for RE-GNN's relation-embedding message passing.

Drop-in surface: the sibling packages ``layer`` (REGraphConv, REGATConv, REMixHopConv, ...) and
``dgl`` (graph front) mirror the reference API. This package holds the device graph layout,
the ctypes boundary to libregnn_hip.so and the autograd operators.
"""
from .graph import RelGraph, RelPack, SegPlan  # noqa: F401

