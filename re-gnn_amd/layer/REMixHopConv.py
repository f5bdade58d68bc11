"""REMixHopConv on MI355X — drop-in for layer/REMixHopConv.py:7-94. Relation embeddings enter only
through the weighted-degree norm; each hop is one HIP SpMM (copy_u) with the pre/post norm fused.
The reference's final propagate (its output is never read, :78-82 on the last j) is skipped."""
import torch
import torch.nn as nn
from torch.nn import init

from regnn_hip import ops

from ._common import relgraph, relation_table


class REMixHopConv(nn.Module):
    def __init__(self, num_etypes, scaling_factor, in_feats, out_feats, p=[0, 1, 2], dropout=0,
                 activation=None, batchnorm=False):
        super().__init__()
        self.in_dim = in_feats
        self.out_dim = out_feats
        self.p = p
        self.activation = activation
        self.batchnorm = batchnorm
        self.dropout = nn.Dropout(dropout)
        self.edge_weight = nn.Parameter(torch.Tensor(num_etypes, 1), requires_grad=True)
        self.alpha = scaling_factor
        if self.batchnorm:
            self.bn = nn.BatchNorm1d(out_feats * len(p))
        self.weights = nn.ModuleDict(
            {str(j): nn.Linear(in_feats, out_feats, bias=False) for j in p})
        self.reset_parameters()

    def reset_parameters(self):
        if self.batchnorm:
            self.bn.reset_parameters()
        for j in self.p:
            self.weights[str(j)].reset_parameters()
        init.constant_(self.edge_weight, 1.0 / self.alpha)

    def forward(self, graph, feats, e_feat):
        rg = relgraph(graph, feats.device)
        pack = rg.rel_pack(e_feat, num_rel=self.edge_weight.shape[0])
        tab = relation_table(self.edge_weight, self.alpha)             # :50-55
        norm = ops.degree_norm(rg, pack, tab)                           # :58-64
        max_j = max(self.p) + 1
        outputs = []
        for j in range(max_j):                                          # :72
            if j in self.p:
                outputs.append(self.weights[str(j)](feats))             # :74-76
            if j < max_j - 1:
                feats = ops.re_spmm(rg, feats, pre=norm, post=norm)     # :78-82 (copy_u)
        final = torch.cat(outputs, dim=1)                               # :84
        if self.batchnorm:
            final = self.bn(final)
        if self.activation is not None:
            final = self.activation(final)
        return self.dropout(final)                                      # :92
