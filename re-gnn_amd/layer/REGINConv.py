"""REGINConv on MI355X — drop-in for layer/REGINConv.py:7-66 (sum aggregation, deg^-1 post-norm)."""
import torch as th
from torch import nn

from dgl.utils import expand_as_pair
from regnn_hip import ops

from ._common import relgraph, relation_table


class REGINConv(nn.Module):
    def __init__(self, num_etypes, scaling_factor, apply_func=None, aggregator_type='sum',
                 init_eps=0, learn_eps=False, activation=None):
        super().__init__()
        self.apply_func = apply_func
        self._aggregator_type = aggregator_type
        self.activation = activation
        if aggregator_type not in ('sum', 'max', 'mean'):
            raise KeyError('Aggregator type {} not recognized.'.format(aggregator_type))
        if learn_eps:
            self.eps = th.nn.Parameter(th.FloatTensor([init_eps]))
        else:
            self.register_buffer('eps', th.FloatTensor([init_eps]))
        self.edge_weight = nn.Parameter(th.Tensor(num_etypes, 1), requires_grad=True)
        self.alpha = scaling_factor
        self.reset_parameters()

    def reset_parameters(self):
        if self.apply_func is not None:
            self.apply_func.reset_parameters()
        nn.init.constant_(self.edge_weight, 1.0 / self.alpha)

    def forward(self, graph, feat, e_feat):
        # the reference reduces with fn.sum whatever aggregator_type names: its `_reducer`
        # (layer/REGINConv.py:40) is never used, so 'max' / 'mean' also sum here
        rg = relgraph(graph, feat.device)
        pack = rg.rel_pack(e_feat, num_rel=self.edge_weight.shape[0])
        tab = relation_table(self.edge_weight, self.alpha)
        norm = ops.degree_norm(rg, pack, tab, power=-1.0)
        feat_src, _ = expand_as_pair(feat, graph)
        rst = ops.re_spmm(rg, feat_src, tab, pack, post=norm)
        if self.apply_func is not None:
            rst = self.apply_func(rst)
        if self.activation is not None:
            rst = self.activation(rst)
        return rst
