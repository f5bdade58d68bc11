"""REGATConv on MI355X — drop-in for layer/REGATConv.py:10-100. The u_add_v SDDMM + relation bias +
LeakyReLU + per-destination edge softmax is one HIP kernel (forward and backward), the per-head
aggregation another, the per-head el/er dots a third; torch does the fc projection (hipBLASLt)."""
import torch as th
from torch import nn
from torch.nn import init

from dgl.nn.pytorch.utils import Identity
from regnn_hip import ops

from ._common import relgraph, relation_table


class REGATConv(nn.Module):
    def __init__(self, num_etypes, scaling_factor, in_feats, out_feats, num_heads, feat_drop=0.,
                 attn_drop=0., negative_slope=0.2, residual=False, activation=None,
                 use_weight=True):
        super().__init__()
        self.num_etypes = num_etypes
        self.num_heads = num_heads
        self.in_feats = in_feats
        self.out_feats = out_feats
        self.use_weight = use_weight
        if self.use_weight:
            self.fc = nn.Linear(in_feats, out_feats * num_heads, bias=False)
        else:
            self.fc = nn.Identity()
        self.attn_l = nn.Parameter(th.FloatTensor(size=(1, num_heads, out_feats)))
        self.attn_r = nn.Parameter(th.FloatTensor(size=(1, num_heads, out_feats)))
        self.feat_drop = nn.Dropout(feat_drop)
        self.attn_drop = nn.Dropout(attn_drop)
        self.leaky_relu = nn.LeakyReLU(negative_slope)
        self.edge_weight = nn.Parameter(th.Tensor(self.num_etypes, self.num_heads),
                                        requires_grad=True)
        self.alpha = scaling_factor
        if residual:
            if in_feats != out_feats:
                self.res_fc = nn.Linear(in_feats, num_heads * out_feats, bias=False)
            else:
                self.res_fc = Identity()
        else:
            self.register_buffer('res_fc', None)
        self.reset_parameters()
        self.activation = activation

    def reset_parameters(self):
        gain = nn.init.calculate_gain('relu')
        if self.use_weight:
            nn.init.xavier_normal_(self.fc.weight, gain=gain)
        nn.init.xavier_normal_(self.attn_l, gain=gain)
        nn.init.xavier_normal_(self.attn_r, gain=gain)
        if isinstance(self.res_fc, nn.Linear):
            nn.init.xavier_normal_(self.res_fc.weight, gain=gain)
        init.constant_(self.edge_weight, 1.0 / self.alpha)

    def forward(self, graph, feat, edge_feats=None):
        rg = relgraph(graph, feat.device)
        h = self.feat_drop(feat)                                                   # :66
        ft = self.fc(h).view(-1, self.num_heads, self.out_feats)                   # :67
        el, er = ops.attn_dots(ft, self.attn_l, self.attn_r)                       # :68-69
        tab = pack = None
        if edge_feats is not None:
            tab = relation_table(self.edge_weight, self.alpha)                     # :72-74
            pack = rg.rel_pack(edge_feats, num_rel=self.num_etypes)
        slope = self.leaky_relu.negative_slope
        if self.training and self.attn_drop.p > 0:
            a = ops.gat_attention(rg, el, er, tab, pack, slope)                    # :80-88
            a = self.attn_drop(a)                                                  # :88
            rst = ops.head_spmm(rg, a, ft)                                         # :90-92
        else:
            # no attention dropout: scores, softmax and aggregation in one pass (:80-92)
            rst = ops.gat_fused(rg, el, er, ft, tab, pack, slope, attn_l=self.attn_l)
        if self.res_fc is not None:
            resval = self.res_fc(h).view(h.shape[0], -1, self.out_feats)           # :94-96
            rst = rst + resval
        if self.activation:
            rst = self.activation(rst)                                             # :98-99
        return rst
