"""REGATv2Conv on MI355X — drop-in for layer/REGATv2Conv.py:12-163. The
GATv2 score <attn, LeakyReLU(fs[u] + fd[v])> is one HIP SDDMM that never forms the (E, H, D)
tensor (regnn_gatv2_score_*), the relation bias and per-destination softmax one HIP pass
(regnn_edge_softmax_*), and the aggregation the HIP per-head SpMM."""
import torch as th
from torch import nn

from dgl.base import DGLError
from dgl.nn.pytorch.utils import Identity
from dgl.utils import expand_as_pair
from regnn_hip import ops

from ._common import relgraph, relation_table


class REGATv2Conv(nn.Module):
    def __init__(self, num_etypes, scaling_factor, in_feats, out_feats, num_heads, feat_drop=0.,
                 attn_drop=0., negative_slope=0.2, residual=False, activation=None,
                 allow_zero_in_degree=False, bias=True, share_weights=False, use_weight=True):
        super().__init__()
        self.num_etypes = num_etypes
        self._num_heads = num_heads
        self._in_src_feats, self._in_dst_feats = expand_as_pair(in_feats)
        self._out_feats = out_feats
        self._allow_zero_in_degree = allow_zero_in_degree
        self.use_weight = use_weight
        if self.use_weight:
            self.fc_src = nn.Linear(self._in_src_feats, out_feats * num_heads, bias=bias)
            if isinstance(in_feats, tuple):
                self.fc_dst = nn.Linear(self._in_dst_feats, out_feats * num_heads, bias=bias)
            elif share_weights:
                self.fc_dst = self.fc_src
            else:
                self.fc_dst = nn.Linear(self._in_src_feats, out_feats * num_heads, bias=bias)
        else:
            self.fc_src = nn.Identity()
            self.fc_dst = nn.Identity()
        self.attn = nn.Parameter(th.FloatTensor(size=(1, num_heads, out_feats)))
        self.feat_drop = nn.Dropout(feat_drop)
        self.attn_drop = nn.Dropout(attn_drop)
        self.leaky_relu = nn.LeakyReLU(negative_slope)
        self.edge_weight = nn.Parameter(th.Tensor(self.num_etypes, num_heads), requires_grad=True)
        self.alpha = scaling_factor
        if residual:
            if self._in_dst_feats != out_feats:
                self.res_fc = nn.Linear(self._in_dst_feats, num_heads * out_feats, bias=bias)
            else:
                self.res_fc = Identity()
        else:
            self.register_buffer('res_fc', None)
        self.activation = activation
        self.share_weights = share_weights
        self.bias = bias
        self.reset_parameters()

    def reset_parameters(self):
        gain = nn.init.calculate_gain('relu')
        if self.use_weight:
            nn.init.xavier_normal_(self.fc_src.weight, gain=gain)
            if self.bias:
                nn.init.constant_(self.fc_src.bias, 0)
            if not self.share_weights:
                nn.init.xavier_normal_(self.fc_dst.weight, gain=gain)
                if self.bias:
                    nn.init.constant_(self.fc_dst.bias, 0)
        nn.init.xavier_normal_(self.attn, gain=gain)
        if isinstance(self.res_fc, nn.Linear):
            nn.init.xavier_normal_(self.res_fc.weight, gain=gain)
            if self.bias:
                nn.init.constant_(self.res_fc.bias, 0)
        nn.init.constant_(self.edge_weight, 1.0 / self.alpha)

    def set_allow_zero_in_degree(self, set_value):
        self._allow_zero_in_degree = set_value

    def forward(self, graph, feat, edge_feats=None, get_attention=False):
        if not self._allow_zero_in_degree and (graph.in_degrees() == 0).any():
            raise DGLError('There are 0-in-degree nodes in the graph; add self loops or set '
                           'allow_zero_in_degree=True')
        rg = relgraph(graph, feat[0].device if isinstance(feat, tuple) else feat.device)
        H, D = self._num_heads, self._out_feats
        if isinstance(feat, tuple):
            h_src, h_dst = self.feat_drop(feat[0]), self.feat_drop(feat[1])
            feat_src = self.fc_src(h_src).view(-1, H, D)
            feat_dst = self.fc_dst(h_dst).view(-1, H, D)
        else:
            h_src = h_dst = self.feat_drop(feat)
            feat_src = self.fc_src(h_src).view(-1, H, D)
            feat_dst = feat_src if self.share_weights else self.fc_dst(h_src).view(-1, H, D)
        s = ops.gatv2_scores(rg, feat_src, feat_dst, self.attn,                    # :139-141
                             self.leaky_relu.negative_slope)
        tab = pack = None
        if edge_feats is not None:
            tab = relation_table(self.edge_weight, self.alpha)                     # :144-149
            pack = rg.rel_pack(edge_feats, num_rel=self.num_etypes)
        a = self.attn_drop(ops.edge_softmax_logits(rg, s, tab, pack))              # :152
        rst = ops.head_spmm(rg, a, feat_src)                                       # :154-156
        if self.res_fc is not None:
            rst = rst + self.res_fc(h_dst).view(h_dst.shape[0], -1, D)             # :158-160
        if self.activation:
            rst = self.activation(rst)
        if get_attention:
            a_e = th.empty_like(a)
            a_e[rg.csr_eid] = a                                                    # caller order
            return rst, a_e.unsqueeze(-1)
        return rst
