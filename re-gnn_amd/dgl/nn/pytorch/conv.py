"""Homogeneous DGL baselines (model/GCN.py, model/GAT.py) are outside the relation-embedding hot
path; the names exist so that ``model/__init__.py`` imports, and constructing them says so."""
import torch.nn as nn


class GraphConv(nn.Module):
    def __init__(self, *args, **kwargs):
        raise NotImplementedError("dgl.nn.pytorch.conv.GraphConv (homogeneous GCN baseline, "
                                  "run_gnn.py) is not part of the RE-GNN MI355X build")


class GATConv(GraphConv):
    pass
