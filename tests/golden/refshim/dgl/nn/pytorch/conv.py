"""Import-only stubs: model/GCN.py and model/GAT.py import these names eagerly."""
import torch.nn as nn


class GraphConv(nn.Module):
    def __init__(self, *a, **k):
        raise NotImplementedError("homogeneous GraphConv is out of scope for the golden shim")


class GATConv(GraphConv):
    pass
