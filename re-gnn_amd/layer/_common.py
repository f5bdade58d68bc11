"""Shared helpers of the drop-in layers."""
import torch
import torch.nn.functional as F


def relgraph(graph, device):
    """the device CSR/CSC layout behind a dgl-front graph (or a RelGraph passed directly)."""
    if hasattr(graph, "relgraph"):
        return graph.relgraph(device)
    if hasattr(graph, "csr_ptr"):
        return graph
    raise TypeError(f"expected a dgl.DGLGraph from the regnn front, got {type(graph)}")


def relation_table(edge_weight, alpha):
    """LeakyReLU(alpha * w) with nn.LeakyReLU()'s default slope 0.01 (layer/REGraphConv.py:58-60)."""
    return F.leaky_relu(edge_weight * alpha, 0.01)
