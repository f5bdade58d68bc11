"""REGraphConv on MI355X — drop-in for layer/REGraphConv.py:7-106 (same constructor, forward
signature, parameters and state_dict keys). The weighted degree, the normalised relation-weighted
SpMM and their backward run as HIP kernels (regnn_hip.ops); torch does the R-sized relation table
and the optional dense projection (hipBLASLt)."""
import torch as th
from torch import nn
from torch.nn import init

from regnn_hip import ops

from ._common import relgraph, relation_table


class REGraphConv(nn.Module):
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
            self.weight = nn.Parameter(th.Tensor(in_feats, out_feats))
        else:
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

    def forward(self, graph, feat, e_feat, return_embedding=False, pre_dropout=0.0,
                project=None, emit=None, drop_seed=None):
        """``pre_dropout`` (not in the reference signature, default off): the probability of a
        caller's nn.Dropout applied to ``feat`` just before this layer (model/REGCN.py:43), so
        both dropouts fuse into the aggregation's gather when it reads ``feat`` directly.

        ``project`` (not in the reference signature): instead of ``feat``, a callable
        ``project(norm, drop) -> (feat, norm * drop(feat))`` for a weightless normalised layer:
        the caller's producer of ``feat`` forms the pre-scaled rows the aggregation gathers
        (nets.REGCN with ops.type_project_prescale); results are the same.

        ``emit`` (not in the reference signature): ``(scale, drop)`` of a next weightless layer
        that reads this layer's output as is; the call then returns ``(rst, xs)`` with
        ``xs = drop(scale * rst)`` formed in the aggregation's epilogue (None where it cannot
        be), which that layer takes through its ``project`` hook.

        ``drop_seed`` (not in the reference signature): the device seed of this layer's fused
        dropout (ops.drop_request), drawn per call when None."""
        if emit is not None and (self.weight is not None or self.activation is not None):
            return self.forward(graph, feat, e_feat, return_embedding, pre_dropout, project,
                                drop_seed=drop_seed), None
        if project is not None:
            return self._forward_projected(graph, e_feat, project, pre_dropout, emit, drop_seed)
        rg = relgraph(graph, feat.device)
        pack = rg.rel_pack(e_feat, num_rel=self.edge_weight.shape[0])
        keep = 1.0
        if self.training:
            keep = (1.0 - self.feat_dropout.p) * (1.0 - pre_dropout)
        direct = self.weight is None or self.in_feats <= self.out_feats  # SpMM reads feat as is
        p_drop = 0.0
        if keep < 1.0 and keep > 0.0 and direct and ops.dropout_fusable(feat):
            p_drop = 1.0 - keep                                          # :56 fused in the gather
        else:
            if self.training and pre_dropout:
                feat = th.nn.functional.dropout(feat, pre_dropout, training=True)
            feat = self.feat_dropout(feat)                               # :56
        tab = relation_table(self.edge_weight, self.alpha)               # :58-61 (folded: no E-sized ew)
        norm = ops.degree_norm(rg, pack, tab) if self.norm else None     # :66-75
        if self.in_feats > self.out_feats:                               # :78
            if self.weight is not None:
                feat = th.matmul(feat, self.weight)                      # :81
            rst = ops.re_spmm(rg, feat, tab, pack, pre=norm, post=norm,  # :76,84-86,97-101
                              bias=self.bias, dropout=p_drop, drop_seed=drop_seed)
        elif self.weight is None:
            rst = ops.re_spmm(rg, feat, tab, pack, pre=norm, post=norm, bias=self.bias,
                              dropout=p_drop, emit=emit, drop_seed=drop_seed)
            if emit is not None:
                return rst                                               # (rst, xs)
        else:
            # diag(norm) (A X) W == (diag(norm) A X) W: post-scale fused into the SpMM epilogue
            rst = th.matmul(ops.re_spmm(rg, feat, tab, pack, pre=norm, post=norm,
                                        dropout=p_drop, drop_seed=drop_seed), self.weight)
            if self.bias is not None:
                rst = rst + self.bias
        if self.activation is not None:
            rst = self.activation(rst)                                   # :103-104
        return rst

    def _forward_projected(self, graph, e_feat, project, pre_dropout=0.0, emit=None,
                           drop_seed=None):
        if self.weight is not None or not self.norm:
            raise ValueError("project= needs a weightless, normalised layer")
        dev = self.edge_weight.device
        rg = relgraph(graph, dev)
        pack = rg.rel_pack(e_feat, num_rel=self.edge_weight.shape[0])
        p_drop = 0.0
        if self.training:                                                # :56 (+ caller's)
            p_drop = 1.0 - (1.0 - self.feat_dropout.p) * (1.0 - pre_dropout)
        tab = relation_table(self.edge_weight, self.alpha)               # :58-61
        norm = ops.degree_norm(rg, pack, tab)                            # :66-75
        drop = ops.drop_request(p_drop, dev, drop_seed) if 0.0 < p_drop < 1.0 else None
        feat, xs = project(norm.detach(), drop)                          # :56,73-76 fused
        if p_drop >= 1.0:
            feat, xs = th.zeros_like(feat), None
        rst = ops.re_spmm(rg, feat, tab, pack, pre=norm, post=norm, bias=self.bias,
                          dropout=p_drop if drop is not None else 0.0,
                          drop_seed=None if drop is None else drop[0], prescaled=xs, emit=emit)
        if emit is not None:
            return rst                                                   # (rst, xs)
        if self.activation is not None:
            rst = self.activation(rst)                                   # :103-104
        return rst
