"""RESAGEConv on MI355X — drop-in for layer/RESAGEConv.py:8-114 (deg^-1 pre-norm, root term).
Not a BASELINE config; it rides on the same HIP degree + SpMM operators."""
import torch as th
from torch import nn
from torch.nn import init

from regnn_hip import ops

from ._common import relgraph, relation_table


class RESAGEConv(nn.Module):
    def __init__(self, num_etypes, scaling_factor, in_feats, out_feats, norm=True, bias=True,
                 activation=None, weight=True, dropout=0.):
        super().__init__()
        self.in_feats = in_feats
        self.out_feats = out_feats
        self.norm = norm
        self.dropout = dropout
        self.edge_weight = nn.Parameter(th.Tensor(num_etypes, 1), requires_grad=True)
        self.alpha = scaling_factor
        if weight:
            # the reference declares weight_root but its forward uses self.weight for the root
            # term (:60-61); both exist so state_dicts match
            self.weight_root = nn.Parameter(th.Tensor(in_feats, out_feats))
            self.weight = nn.Parameter(th.Tensor(in_feats, out_feats))
        else:
            self.register_parameter('weight_root', None)
            self.register_parameter('weight', None)
        if bias:
            self.bias = nn.Parameter(th.Tensor(out_feats))
        else:
            self.register_parameter('bias', None)
        self.reset_parameters()
        self.feat_dropout = nn.Dropout(p=self.dropout)
        self.activation = activation

    def reset_parameters(self):
        if self.weight is not None:
            init.xavier_uniform_(self.weight)
        if self.bias is not None:
            init.zeros_(self.bias)
        init.constant_(self.edge_weight, 1.0 / self.alpha)

    def forward(self, graph, feat, e_feat):
        rg = relgraph(graph, feat.device)
        pack = rg.rel_pack(e_feat, num_rel=self.edge_weight.shape[0])
        feat = self.feat_dropout(feat)
        feat_root = th.matmul(feat, self.weight) if self.weight_root is not None else feat
        tab = relation_table(self.edge_weight, self.alpha)
        norm = ops.degree_norm(rg, pack, tab, power=-1.0) if self.norm else None
        if self.in_feats > self.out_feats:
            if self.weight is not None:
                feat = th.matmul(feat, self.weight)
            rst = ops.re_spmm(rg, feat, tab, pack, pre=norm)
        else:
            rst = ops.re_spmm(rg, feat, tab, pack, pre=norm)
            if self.weight is not None:
                rst = th.matmul(rst, self.weight)
        rst = rst + feat_root
        if self.bias is not None:
            rst = rst + self.bias
        if self.activation is not None:
            rst = self.activation(rst)
        return rst
