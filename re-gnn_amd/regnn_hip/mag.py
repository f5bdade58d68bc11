"""ogbn-mag neighbour-sampled path on MI355X: mag ``REGCNConv`` (mag/regnn_layers.py:24-150), the
``REGNN`` model (mag/regnn_ns.py:216-369) and a data-parallel train step with a flat-bucket RCCL
gradient all-reduce (inserted between mag/regnn_ns.py:406 and :407).

The sampled block's aggregation (PyG propagate with aggr='mean', message ew * x_j, update +bias)
runs as one HIP SpMM with the relation table, the 1/in-count scale and the bias fused; its
backward is the fused transposed SpMM + relation-bin SDDMM.
"""
import os

import torch
import torch.distributed as dist
import torch.nn.functional as F
from torch.nn import Linear, ModuleDict, ModuleList, Parameter, ParameterDict, init

from . import ops
from .graph import RelGraph


def make_block(edge_index, edge_type, target_node_type, n_src, n_dst, num_edge_types,
               self_loop_type=2):
    """device CSR/CSC of a sampled bipartite block, self loops appended for the targets with
    type ntype + num_edge_types (mag/regnn_layers.py:90-96). Returns (RelGraph, RelPack)."""
    src, dst = edge_index[0].to(torch.int64), edge_index[1].to(torch.int64)
    et = edge_type.to(torch.int64)
    if self_loop_type == 2:
        loop = torch.arange(n_dst, device=src.device)
        src = torch.cat([src, loop])
        dst = torch.cat([dst, loop])
        et = torch.cat([et, target_node_type.to(torch.int64) + num_edge_types])
    rg = RelGraph(src, dst, n_src, src.device, num_dst=n_dst)
    pack = rg.rel_pack(et + 1)
    return rg, pack


class REGCNConv(torch.nn.Module):
    """mag/regnn_layers.py:24-150 (same constructor, parameters and forward signature)."""

    def __init__(self, in_channels, out_channels, num_node_types, num_edge_types,
                 scaling_factor=100., dropout=0., use_softmax=False, residual=False,
                 use_norm=None, self_loop_type=1, no_re=False):
        super().__init__()
        self.in_channels, self.out_channels = in_channels, out_channels
        self.num_node_types, self.num_edge_types = num_node_types, num_edge_types
        self.use_softmax = use_softmax
        self.dropout, self.residual, self.use_norm = dropout, residual, use_norm
        self.self_loop_type = self_loop_type
        self.weight = Parameter(torch.Tensor(in_channels, out_channels))
        if self.residual:
            self.weight_root = self.weight        # shared, as in the reference (:51)
        self.bias = Parameter(torch.Tensor(out_channels))
        rw_dim = num_edge_types if self_loop_type in (1, 3) else num_edge_types + num_node_types
        self.relation_weight = Parameter(torch.Tensor(rw_dim), requires_grad=not no_re)
        self.scaling_factor = scaling_factor
        if self.use_norm == 'bn':
            self.norm = torch.nn.BatchNorm1d(out_channels)
        elif self.use_norm == 'ln':
            self.norm = torch.nn.LayerNorm(out_channels)
        self.reset_parameters()

    def reset_parameters(self):
        init.xavier_uniform_(self.weight)
        if self.residual:
            # weight_root IS weight: the reference draws it a second time (:73-74), so a seeded
            # model's weights (and the RNG stream after them) match the reference's only with it
            init.xavier_uniform_(self.weight_root)
        init.zeros_(self.bias)
        init.constant_(self.relation_weight, 1.0 / self.scaling_factor)
        if self.use_norm in ('bn', 'ln'):
            self.norm.reset_parameters()

    def forward(self, x, edge_index, edge_type=None, target_node_type=None,
                return_weights=False):
        x_src, x_target = x
        tab = F.leaky_relu(self.relation_weight * self.scaling_factor)           # :110-111
        # mean of ew * x_j over in-edges incl. self loops, + bias (:113,129,142-148); the
        # use_softmax / degree-normalised ew of :116-126 is computed there but propagate() gets
        # the raw edge_weight, so neither changes the output (only return_weights shows ew)
        if getattr(edge_index, "is_ns_block", False):             # device-sampled block
            # aggregate first, project second: mean_e(ew x_j) W = mean_e(ew (x_j W)) (the
            # reference projects every source row first, :101-107), so the GEMM and its two
            # backward GEMMs run over the block's targets, not its sources (~11x fewer rows at
            # fan-out [25, 20]); the residual x_target W folds into the same product (:104,131)
            agg = ops.ns_spmm(edge_index, x_src, tab)
            if self.residual:
                agg = agg + x_target
            out = ops.mm(agg, self.weight, self.bias)
            if self.use_norm in ('bn', 'ln'):
                out = self.norm(out)                                             # :134-135
            if return_weights:
                return out, self._edge_weights(edge_index, edge_type, target_node_type, tab,
                                               x_target.shape[0]), tab
            return out
        xs = ops.mm(x_src, self.weight)                                          # :102
        if isinstance(edge_index, tuple):           # pre-built (RelGraph, RelPack) block
            rg, pack = edge_index
        else:
            rg, pack = make_block(edge_index, edge_type, target_node_type, x_src.shape[0],
                                  x_target.shape[0], self.num_edge_types, self.self_loop_type)
        out = ops.re_spmm(rg, xs, tab, pack, post=rg.inv_in_count(), bias=self.bias)
        if self.residual:
            out = out + ops.mm(x_target, self.weight)                            # :104,131-132
        if self.use_norm in ('bn', 'ln'):
            out = self.norm(out)                                                 # :134-135
        if return_weights:
            return out, self._edge_weights(edge_index, edge_type, target_node_type, tab,
                                           x_target.shape[0]), tab
        return out

    def forward_act(self, x_src, x_target, blk, p, state, layer, tab=None):
        """forward() on a device-sampled block followed by the model's relu and dropout, the
        bias / LayerNorm / relu / dropout as one launch (ops.wide_ln_act). tab: this layer's
        relation table when the caller formed it (ops.rel_tabs)."""
        if tab is None:
            tab = ops.rel_tab(self.relation_weight, self.scaling_factor)        # :110-111
        agg = ops.ns_spmm(blk, x_src, tab)
        if self.residual:
            agg = agg + x_target
        return ops.wide_ln_act(ops.mm(agg, self.weight), self.bias, self.norm, p, state, layer)

    def _edge_weights(self, edge_index, edge_type, target_node_type, tab, n_dst):
        """ew of mag/regnn_layers.py:110-126 per edge in the reference's order (sampled edges,
        then the appended self loops): softmax of tab[type] over each target's in-edges with the
        global max subtracted and + 1e-16 (mag/utils.py:45-57) when use_softmax, else
        tab[type] / weighted in-degree (weighted_degree, mag/utils.py:15-21)."""
        if not isinstance(edge_index, torch.Tensor):
            raise ValueError("return_weights needs the edge_index / edge_type tensors")
        col = edge_index[1].to(torch.int64)
        et = edge_type.to(torch.int64)
        if self.self_loop_type == 2:
            loop = torch.arange(n_dst, device=col.device)
            col = torch.cat([col, loop])
            et = torch.cat([et, target_node_type.to(torch.int64) + self.num_edge_types])
        with torch.no_grad():
            w = tab.detach()[et]
            if self.use_softmax:
                e = (w - w.max()).exp()
                den = torch.zeros(n_dst, dtype=e.dtype, device=e.device).index_add_(0, col, e)
                return e / (den[col] + 1e-16)
            deg = torch.zeros(n_dst, dtype=w.dtype, device=w.device).index_add_(0, col, w)
            return w * deg.pow(-1.0)[col]


def _typed_block(adj, edge_type, ntype_dst, n_id, size, num_edge_types):
    """NSBlock of a sampled Adj (dst-major edge_index, per-target counts) with its relation ids
    from the caller's edge_type (mag/regnn_layers.py:90-99): sampled edges in order, the target's
    self loop last in its row. Device ops only, sizes from the Adj."""
    from .ns import NSBlock
    ei, e_id = adj.edge_index, adj.e_id
    n_src, n_dst = size
    dev = ei.device
    M = ei.shape[1]
    cnt = adj.counts.to(torch.int64) + 1
    ptr = torch.zeros(n_dst + 1, dtype=torch.int64, device=dev)
    torch.cumsum(cnt, 0, out=ptr[1:])
    posn = torch.arange(M, device=dev) + ei[1]
    loop_pos = ptr[1:] - 1
    E = M + n_dst
    idx = torch.empty(E, dtype=torch.int32, device=dev)
    idx[posn] = ei[0].to(torch.int32)
    idx[loop_pos] = torch.arange(n_dst, device=dev, dtype=torch.int32)
    rel = torch.empty(E, dtype=torch.uint8, device=dev)
    rel[posn] = edge_type[e_id].to(torch.uint8)
    rel[loop_pos] = (ntype_dst + num_edge_types).to(torch.uint8)
    inv = (1.0 / cnt.to(torch.float32)).contiguous()
    return NSBlock(ptr.to(torch.int32), idx, rel, None, inv, n_dst, n_src, E, dev)


def _block_of(x_src, x_dst, edge_index, edge_type, target_node_type, num_edge_types,
              self_loop_type):
    if isinstance(edge_index, tuple):           # pre-built (RelGraph, RelPack) block
        return edge_index
    return make_block(edge_index, edge_type, target_node_type, x_src.shape[0], x_dst.shape[0],
                      num_edge_types, self_loop_type)


class REGATConv(torch.nn.Module):
    """mag/regnn_layers.py:153-315 (same constructor, parameters, state_dict and forward).

    Scores LeakyReLU(rw[type] + att_src.x_src[u] + att_dst.x_dst[v]) and the ogbn-mag softmax
    (one global max, + 1e-16, mag/utils.py:45-57) run as HIP kernels (regnn_gat_scores,
    regnn_edge_softmax_fwd; backward regnn_gat_softmax_bwd + segment sums), the aggregation as
    the HIP per-head SpMM."""

    v2 = False

    def __init__(self, in_channels, out_channels, num_node_types, num_edge_types, heads=1,
                 scaling_factor=100., concat=True, negative_slope=0.2, dropout=0.0,
                 residual=False, use_norm=None, self_loop_type=1, no_re=False):
        super().__init__()
        self.in_channels, self.out_channels = in_channels, out_channels
        self.heads, self.concat = heads, concat
        self.negative_slope, self.dropout = negative_slope, dropout
        self.num_node_types, self.num_edge_types = num_node_types, num_edge_types
        self.residual, self.use_norm, self.self_loop_type = residual, use_norm, self_loop_type
        self.out_dim = heads * out_channels if concat else out_channels
        self.lin_src = Linear(in_channels, heads * out_channels, bias=False)
        self.lin_dst = self.lin_src                                          # :189
        self.bias = Parameter(torch.Tensor(self.out_dim))
        rw_dim = num_edge_types if self_loop_type in (1, 3) else num_edge_types + num_node_types
        self.relation_weight = Parameter(torch.Tensor(rw_dim, heads), requires_grad=not no_re)
        self.scaling_factor = scaling_factor
        self._make_att()
        if use_norm == 'bn':
            self.norm = torch.nn.BatchNorm1d(self.out_dim)
        elif use_norm == 'ln':
            self.norm = torch.nn.LayerNorm(self.out_dim)
        self.reset_parameters()

    def _make_att(self):
        self.att_src = Parameter(torch.Tensor(1, self.heads, self.out_channels))
        self.att_dst = Parameter(torch.Tensor(1, self.heads, self.out_channels))

    def _reset_att(self):
        init.xavier_uniform_(self.att_src)
        init.xavier_uniform_(self.att_dst)

    def reset_parameters(self):
        self.lin_src.reset_parameters()
        self.lin_dst.reset_parameters()
        self._reset_att()
        init.zeros_(self.bias)
        init.constant_(self.relation_weight, 1.0 / self.scaling_factor)
        if self.use_norm in ('bn', 'ln'):
            self.norm.reset_parameters()

    def _attention(self, rg, pack, x_src, x_dst, tab):
        a_s = (x_src * self.att_src).sum(dim=-1)                             # :289
        a_d = (x_dst * self.att_dst).sum(dim=-1)                             # :290
        return ops.gat_attention(rg, a_s, a_d, tab, pack, self.negative_slope,
                                 global_max=True)                           # :298-307

    def forward(self, x, edge_index, edge_type=None, target_node_type=None,
                return_weights=False):
        H, C = self.heads, self.out_channels
        if isinstance(x, torch.Tensor):
            x_src = x_dst = self.lin_src(x).view(-1, H, C)
            n_dst = x.shape[0]
        else:
            xs_in, xd_in = x
            x_src = self.lin_src(xs_in).view(-1, H, C)                       # :271-274
            x_dst = self.lin_dst(xd_in).view(-1, H, C)
            n_dst = xd_in.shape[0]
        rg, pack = _block_of(x_src, x_dst, edge_index, edge_type, target_node_type,
                             self.num_edge_types, self.self_loop_type)
        assert rg.n_dst == n_dst
        tab = F.leaky_relu(self.relation_weight * self.scaling_factor)       # :294-295
        a = self._attention(rg, pack, x_src, x_dst, tab)
        out = ops.head_spmm(rg, a, x_src)                                    # propagate :312
        out = out.reshape(-1, H * C) if self.concat else out.mean(dim=1)     # :314-317
        out = out + self.bias                                                # :319
        if self.residual:
            out = out + x_dst.reshape(-1, H * C)                             # :321-322
        if self.use_norm in ('bn', 'ln'):
            out = self.norm(out)                                             # :324-325
        if return_weights:
            ew = torch.empty_like(a)
            if hasattr(rg, "csr_eid"):
                ew[rg.csr_eid] = a                                           # caller edge order
            else:
                ew = a
            return out, ew
        return out


class REGATv2Conv(REGATConv):
    """mag/regnn_layers.py:318-436: score <att, LeakyReLU(x_src[u] + x_dst[v])> + rw[type] (HIP
    GATv2 SDDMM, regnn_gatv2_score_*), the same global-max softmax (regnn_edge_softmax_*)."""

    v2 = True

    def _make_att(self):
        self.att = Parameter(torch.Tensor(1, self.heads, self.out_channels))

    def _reset_att(self):
        init.xavier_uniform_(self.att)

    def _attention(self, rg, pack, x_src, x_dst, tab):
        s = ops.gatv2_scores(rg, x_src, x_dst, self.att, self.negative_slope)  # :399-404
        return ops.edge_softmax_logits(rg, s, tab, pack, global_max=True)     # :407-413


# "auto": layer 0 of a device-block REGNN (regcn, self-loop type 2, feats_type 3) aggregates the
# raw input rows per node type and projects after (REGNN._typed_first_layer); "off": group_input
# over every sampled node first, as the reference orders it (tests compare the two)
TYPED_AGG = {"mode": "auto"}
# "on": at hidden >= 128 the device-block path runs each layer's bias / residual / LayerNorm /
# relu / dropout as one launch each way (ops.wide_ln_act: regnn_wide_ln_fwd / _bwd); "off":
# torch's kernels (A/B, tests)
WIDE_EPI = {"mode": os.environ.get("REGNN_WIDE_EPI", "on")}
# all layers' relation tables from one launch (ops.rel_tabs) on device-sampled blocks
REL_TABS = os.environ.get("REGNN_REL_TABS", "1") != "0"


class REGNN(torch.nn.Module):
    """mag/regnn_ns.py:216-369 for model 'regcn' (feats_type != 2)."""

    def __init__(self, in_channels, hidden_channels, out_channels, num_layers, scaling_factor,
                 dropout, num_feature_dict, num_edge_types, residual=False, no_re=False,
                 use_norm='ln', self_loop_type=2, model='regcn', heads=8, feats_type=3,
                 num_nodes_dict=None, target_node_type=0):
        super().__init__()
        if model not in ('regcn', 'regat', 'regatv2'):
            raise NotImplementedError(model)
        self.model = model
        self.in_channels = in_channels
        self.hidden_dim = hidden_channels if model == 'regcn' else hidden_channels * heads
        self.num_layers, self.dropout = num_layers, dropout
        self.num_node_types = len(num_feature_dict)
        self.num_edge_types = num_edge_types
        self.self_loop_type = self_loop_type
        self.feats_type = feats_type
        self._touched = {}
        if feats_type == 2:
            # learned per-type embeddings for every non-target type (regnn_ns.py:240-245)
            self.emb_dict = ParameterDict({
                str(k): Parameter(torch.Tensor(num_nodes_dict[k], in_channels))
                for k in sorted(set(num_feature_dict) - {target_node_type})})
            self.lin = Linear(in_channels, self.hidden_dim)
        else:
            # created in the reference's order (`for key in set(node_types)`, :248-250): the RNG
            # stream of a seeded construction then matches
            self.lins = ModuleDict({str(k): Linear(num_feature_dict[k], self.hidden_dim)
                                    for k in set(num_feature_dict)})
        if model == 'regcn':                                                # regnn_ns.py:245-270
            convs = [REGCNConv(hidden_channels, hidden_channels, self.num_node_types,
                               num_edge_types, scaling_factor, dropout=dropout,
                               residual=residual, use_norm=use_norm,
                               self_loop_type=self_loop_type, no_re=no_re)
                     for _ in range(num_layers)]
        else:
            cls = REGATConv if model == 'regat' else REGATv2Conv
            convs = [cls(self.hidden_dim, hidden_channels, self.num_node_types, num_edge_types,
                         heads, scaling_factor, dropout=dropout, residual=residual,
                         use_norm=use_norm, self_loop_type=self_loop_type, no_re=no_re)
                     for _ in range(num_layers)]
        self.convs = ModuleList(convs)
        self.out_lin = Linear(self.hidden_dim, out_channels)
        if use_norm == 'ln':
            self.norm = torch.nn.LayerNorm(self.hidden_dim)   # declared, unused in forward
        elif use_norm == 'bn':
            self.norm = torch.nn.BatchNorm1d(self.hidden_dim)
        self.reset_parameters()

    def reset_parameters(self):
        """mag/regnn_ns.py:284-298, in its order (a seeded model draws the reference's values)."""
        if self.feats_type == 2:
            for emb in self.emb_dict.values():
                init.xavier_uniform_(emb)
            self.lin.reset_parameters()
        else:
            for lin in self.lins.values():
                lin.reset_parameters()
        for conv in self.convs:
            conv.reset_parameters()
        self.out_lin.reset_parameters()
        if hasattr(self, "norm"):
            self.norm.reset_parameters()

    def embedding_tables(self):
        """[(table parameter, local rows the last forward read)] of the feats_type-2 tables."""
        if self.feats_type != 2:
            return []
        if self._touched is None:                    # formed on demand (boolean masks sync)
            nt, li = self._batch_rows
            self._touched = {k: li[nt == int(k)] for k in self.emb_dict}
        return [(emb, self._touched.get(k)) for k, emb in self.emb_dict.items()]

    def _type_tables(self, x_dict):
        """the input tables indexed by node type (feats_type 2: the learned embeddings for the
        non-target types), or None when a key lies outside 0..T-1."""
        T = self.num_node_types
        keys = set(x_dict) | ({int(k) for k in self.emb_dict} if self.feats_type == 2 else set())
        if not keys <= set(range(T)):
            return None
        tabs = [x_dict.get(k) for k in range(T)]
        if self.feats_type == 2:
            for k, emb in self.emb_dict.items():
                tabs[int(k)] = emb
        return tabs

    def group_input(self, x_dict, node_type, local_node_idx, n_id=None):
        """mag/regnn_ns.py:300-326 without per-type masks or host syncs: feats_type 2 gathers
        every node's row from its type's table in one launch (ops.typed_gather) before the shared
        Linear; otherwise each node's row goes through its own type's Linear in one gather-fused
        MFMA launch over the type-sorted rows (ops.typed_linear). Other shapes: one GEMM against
        all types' weights + a per-node pick."""
        tabs = self._type_tables(x_dict)
        on_dev = tabs is not None and all(t is None or (t.is_cuda and t.dtype == torch.float32
                                                        and t.dim() == 2) for t in tabs)
        widths = {t.shape[1] for t in tabs if t is not None} if on_dev else set()
        if self.feats_type == 2 and len(widths) == 1 and widths.pop() % 4 == 0:
            t = ops.typed_gather(tabs, node_type, local_node_idx, n_id)
            self._batch_rows = ((node_type, local_node_idx) if n_id is None else
                                (node_type[n_id], local_node_idx[n_id]))
            self._touched = None
            return self.lin(t)
        if self.feats_type != 2 and on_dev and all(t is not None for t in tabs):
            Ws = [self.lins[str(k)].weight for k in range(len(tabs))]
            bs = [self.lins[str(k)].bias for k in range(len(tabs))]
            if ops.typed_linear_fusable(tabs, Ws, bs):
                return ops.typed_linear(tabs, Ws, bs, node_type, local_node_idx, n_id)
        if n_id is not None:
            node_type, local_node_idx = node_type[n_id], local_node_idx[n_id]
        if self.feats_type == 2:
            # raw target features + learned embeddings of the other types, one shared Linear
            # (regnn_ns.py:306-315); each table's rows read here are recorded for the
            # sparse-row gradient all-reduce
            t = torch.zeros(node_type.numel(), self.in_channels, device=node_type.device)
            for key, x in x_dict.items():
                idx = torch.nonzero(node_type == key).flatten()
                t[idx] = x[local_node_idx[idx]].to(t.device)
            self._touched = {}
            for key, emb in self.emb_dict.items():
                idx = torch.nonzero(node_type == int(key)).flatten()
                rows = local_node_idx[idx]
                self._touched[key] = rows
                t = t.index_copy(0, idx, emb[rows])
            return self.lin(t)
        keys = sorted(x_dict)
        dims = {x_dict[k].shape[1] for k in keys}
        if len(dims) == 1 and keys == list(range(len(keys))):
            table, offs = self._feature_table(x_dict, keys)
            X = table[offs[node_type] + local_node_idx]
            Wc = torch.cat([self.lins[str(k)].weight for k in keys], 0)
            bc = torch.cat([self.lins[str(k)].bias for k in keys], 0)
            Y = torch.addmm(bc, X, Wc.t()).view(X.shape[0], len(keys), self.hidden_dim)
            return Y[torch.arange(X.shape[0], device=X.device), node_type]
        h = torch.zeros(node_type.numel(), self.hidden_dim, device=node_type.device)
        for key, x in x_dict.items():
            mask = node_type == key
            h[mask] = self.lins[str(key)](x[local_node_idx[mask]])
        return h

    def _feature_table(self, x_dict, keys):
        sig = tuple((k, x_dict[k].data_ptr(), x_dict[k].shape[0]) for k in keys)
        cache = getattr(self, "_ftab", None)
        if cache is None or cache[0] != sig:
            table = torch.cat([x_dict[k] for k in keys], 0)
            sizes = torch.tensor([0] + [x_dict[k].shape[0] for k in keys[:-1]])
            offs = torch.cumsum(sizes, 0).to(table.device)
            self._ftab = cache = (sig, table, offs)
        return cache[1], cache[2]

    def typed_first_layer_ok(self, x_dict):
        """True when _typed_first_layer takes layer 0 of a device-block batch (NSTrainer then lets
        the sampler's last hop run meta-only: nothing reads its sources' local ids)."""
        if (TYPED_AGG["mode"] == "off" or self.model != 'regcn' or self.feats_type == 2 or
                self.self_loop_type != 2):
            return False
        tabs = self._type_tables(x_dict)
        return (tabs is not None and ops.ns_typed_agg_ok(tabs) and
                self.convs[0].relation_weight.numel() <= 256)

    def _wide_epi(self, blk):
        """(dropout p, state) when the device-block layers may run the fused wide epilogue
        (ops.wide_ln_act), else None."""
        if (WIDE_EPI["mode"] == "off" or self.model != 'regcn' or self.hidden_dim < 128 or
                self.hidden_dim not in ops.WIDE_LN_WIDTHS or
                any(c.use_norm != 'ln' for c in self.convs)):
            return None
        p = float(self.dropout) if self.training else 0.0
        state = getattr(blk, "state", None)
        if p > 0 and state is None:
            return None
        return p, state

    def _typed_first_layer(self, n_id, x_dict, adjs, node_type, local_node_idx, epi=None,
                           tab=None):
        """layer 0 over a device block with group_input folded in (None: not applicable).

        The reference runs every sampled node's raw row through its type's Linear
        (mag/regnn_ns.py:300-326), then x_src @ W and the relation-weighted mean
        (mag/regnn_layers.py:101-148). All three are linear, so
            a_v = inv_v sum_t (S_vt W_t^T + w_vt b_t) W_0 + bias,
        S_vt = sum_{e in v, type t} tab[r_e] x_raw[src_e] (ops.ns_typed_agg: one read of each
        sampled raw row, no per-node projection) and the composed W_t^T W_0 runs over the
        block's target rows only (~13 k of ~280 k sampled rows at fan-out [25, 20])."""
        if (TYPED_AGG["mode"] == "off" or self.model != 'regcn' or self.feats_type == 2 or
                self.self_loop_type != 2 or not adjs):
            return None
        edge_index, _e_id, _size = adjs[0]
        blk = edge_index if getattr(edge_index, "is_ns_block", False) else \
            getattr(adjs[0], "block", None)
        if blk is None or getattr(blk, "inv", None) is None:
            return None
        tabs = self._type_tables(x_dict)
        if tabs is None or not ops.ns_typed_agg_ok(tabs) or not n_id.is_cuda:
            return None
        conv = self.convs[0]
        if conv.relation_weight.numel() > 256:
            return None
        T, K = len(tabs), int(tabs[0].shape[1])
        if tab is None:
            tab = ops.rel_tab(conv.relation_weight, conv.scaling_factor)       # :110-111
        # [S | w]: the per-type sums and weight sums as one [n, T K + T] operand, so the
        # projection S W_c + w b_c is one GEMM against [W_c; b_c] (products on regnn_gemm_x6:
        # fp32-accurate bf16x6 MFMA; the small composition b_cat W_0 stays on hipBLASLt)
        if getattr(blk, "pre_sums", None) is not None:
            # the sampler formed the per-type input sums ahead (relation slots): [S | w | 0] from
            # one read of them, no gather of the sampled raw rows here
            Sw = ops.ns_slot_agg(blk, tab, self.num_edge_types)
        else:
            Sw = ops.ns_typed_agg(blk, tab, n_id, tabs, node_type, local_node_idx, ext=True)
        lins = [self.lins[str(t)] for t in range(T)]
        n = blk.n_dst
        # [W_c; b_c; 0] = [W_1ᵀ; ..; W_Tᵀ; b_1; ..; b_T; 0] @ W_0: one concatenation and one x6
        # GEMM (the zero rows of the pad a cached constant), forward and backward
        pad = Sw.shape[1] - T * K - T
        zpad = self._zero_rows(pad, conv.weight.shape[0], conv.weight)
        wb_in = torch.cat([lin.weight.t() for lin in lins] +
                          [lin.bias.view(1, -1) for lin in lins] + ([zpad] if pad else []), 0)
        # the block is capacity-sized: its rows past the batch's live targets are zeros, and the
        # GEMMs (forward and both backward products) skip them (live: sizes[hop] on the device)
        agg = ops.mm(Sw, ops.mm(wb_in, conv.weight), live=getattr(blk, "live_rows", None))
        res = None
        if conv.residual:                                                       # :104,131-132
            x_t = self.group_input(x_dict, node_type, local_node_idx, n_id[:n])
            res = ops.mm(x_t, conv.weight)
        if epi is not None and ops.wide_ln_ok(agg, conv.norm, conv.bias):
            # mean + bias + residual, LayerNorm, relu, dropout in one launch (:341-343)
            # (only the block's live rows: without residuals every consumer of layer 0's rows is
            # live-bounded -- layer 1 aggregates sampled rows, the GEMMs take m_live / k_live; a
            # residual reads the first B rows, which a short last batch may leave unformed)
            live = (getattr(blk, "live_rows", None)
                    if not any(getattr(c, "residual", False) for c in self.convs) else None)
            return ops.wide_ln_act(agg, conv.bias, conv.norm, epi[0], epi[1], 0,
                                   rs=blk.inv[:n], res=res, live=live), True
        out = torch.addcmul(conv.bias, agg, blk.inv[:n].view(n, 1))           # mean + bias
        if res is not None:
            out = out + res
        if conv.use_norm in ('bn', 'ln'):
            out = conv.norm(out)                                                # :134-135
        return out, False

    def _zero_rows(self, rows, cols, like):
        """a cached [rows, cols] zero block (no fill launch per step)"""
        z = getattr(self, "_zrows", None)
        if z is None or z.shape != (rows, cols) or z.device != like.device:
            z = self._zrows = like.new_zeros(rows, cols)
        return z

    def forward(self, n_id, x_dict, adjs, edge_type, node_type, local_node_idx, logits=False,
                features=False):
        """-> log_softmax of out_lin (mag/regnn_ns.py:346); logits=True: out_lin's raw output
        (a caller that forms the loss itself, e.g. NSTrainer with ops.softmax_xent);
        features=True: the last layer's output, before out_lin (NSTrainer with ops.ns_lin_xent)."""
        blk0 = tuple(adjs[0])[0] if adjs else None
        epi = self._wide_epi(blk0) if getattr(blk0, "is_ns_block", False) else None
        # every layer's relation table in one launch (and one in the backward) on device blocks
        tabs = None
        if REL_TABS and epi is not None and self.model == 'regcn' and 1 <= len(self.convs) <= 4:
            rws = [getattr(c, "relation_weight", None) for c in self.convs]
            alphas = {getattr(c, "scaling_factor", None) for c in self.convs}
            if (all(r is not None and r.is_cuda and r.dtype == torch.float32 and r.dim() == 1
                    for r in rws) and len(alphas) == 1 and None not in alphas):
                tabs = ops.rel_tabs(rws, alphas.pop())
        r = self._typed_first_layer(n_id, x_dict, adjs, node_type, local_node_idx, epi,
                                    tab=None if tabs is None else tabs[0])
        x, acted = (None, False) if r is None else r
        if x is None and adjs and getattr(tuple(adjs[0])[0], "meta_only", False):
            raise RuntimeError("layer 0's block was sampled meta-only (no local source ids): "
                               "only the typed first layer (TYPED_AGG) can read it")
        start = 0
        if x is not None:                      # layer 0 done (group_input folded in)
            if not acted:
                x = F.relu(x)
                x = F.dropout(x, p=self.dropout, training=self.training)
            start = 1
        else:
            x = self.group_input(x_dict, node_type, local_node_idx, n_id)
        for i, adj in enumerate(adjs):
            if i < start:
                continue
            edge_index, e_id, size = adj
            x_target = x[:size[1]]
            blk = edge_index if getattr(edge_index, "is_ns_block", False) else \
                getattr(adj, "block", None)
            if (blk is not None and getattr(blk, "is_ns_block", False) and epi is not None and
                    self.self_loop_type == 2 and ops.wide_ln_ok(x, self.convs[i].norm, self.convs[i].bias)):
                ep = self._wide_epi(blk) or epi
                x = self.convs[i].forward_act(x, x_target, blk, ep[0], ep[1], i,
                                              tab=None if tabs is None else tabs[i])
                continue                       # (relu and dropout applied in the epilogue)
            if blk is not None and self.model == 'regcn' and self.self_loop_type == 2:
                x = self.convs[i]((x, x_target), blk)          # relation ids formed on device
                x = F.relu(x)
                x = F.dropout(x, p=self.dropout, training=self.training)
                continue
            # the targets' node types (only these paths read them: no gather launch otherwise)
            ntype = node_type[n_id[:size[1]]]
            if (self.model == 'regcn' and self.self_loop_type == 2 and
                    getattr(adj, "counts", None) is not None):
                x = self.convs[i]((x, x_target), _typed_block(adj, edge_type, ntype, n_id, size,
                                                              self.num_edge_types))
            else:
                x = self.convs[i]((x, x_target), edge_index, edge_type[e_id], ntype)
            x = F.relu(x)
            x = F.dropout(x, p=self.dropout, training=self.training)
        if features:
            return x
        out = self.out_lin(x)
        return out if logits else out.log_softmax(dim=-1)

    @torch.no_grad()
    def inference(self, x_dict, subgraph_loader, edge_type, node_type, local_node_idx,
                  device=None):
        """mag/regnn_ns.py:348-369: layer-wise full-neighbour inference -> logits of every node.

        ``subgraph_loader`` is the reference's full-neighbour loader (a NeighborSampler with
        sizes=[-1] over all nodes) or the global RelGraph itself. Its batches are row ranges of
        the full graph, so each layer runs as one full-graph aggregation with the layer input
        resident in HBM (regnn_hip/inference.py); ``inference_sharded`` splits the rows over
        data-parallel ranks."""
        rg = getattr(subgraph_loader, "rg", subgraph_loader)
        sizes = getattr(subgraph_loader, "sizes", [-1])
        if list(sizes) != [-1]:
            raise ValueError(f"inference expects a full-neighbour loader (sizes=[-1]), got {sizes}")
        from .inference import ShardedInference
        return ShardedInference(self, rg, edge_type, node_type, local_node_idx).run(x_dict)

    @torch.no_grad()
    def inference_sharded(self, x_dict, rg, edge_type, node_type, local_node_idx, rank, world,
                          gather="logits", group=None):
        """inference() with the destination rows split over ``world`` ranks and one all-gather
        per layer (RCCL over xGMI); gather=None returns only this rank's rows."""
        from .inference import ShardedInference
        return ShardedInference(self, rg, edge_type, node_type, local_node_idx, rank,
                                world).run(x_dict, gather=gather, group=group)


def flat_grad_allreduce(params, world):
    """one SUM all-reduce of every gradient in a flat fp32 bucket, then / world (RCCL over xGMI
    on ROCm devices; gloo on CPU). Sized 0.26-4 MB for the mag configs: latency-bound, one call."""
    grads = [p.grad for p in params if p.grad is not None]
    if world <= 1 or not grads:
        return
    flat = torch.cat([g.reshape(-1) for g in grads])
    dist.all_reduce(flat, op=dist.ReduceOp.SUM)
    flat /= world
    o = 0
    for g in grads:
        n = g.numel()
        g.copy_(flat[o:o + n].view_as(g))
        o += n


def sparse_rows_allreduce(tables, world, group=None):
    """SUM / world all-reduce of embedding-table gradients that are zero outside the rows each
    rank touched (feats_type 2): every rank all-gathers the (row ids, grad
    rows) of the others and adds them in rank order, so the traffic is the touched rows instead
    of the whole table (~154 M parameters at the reference's defaults) and every rank ends with
    the same dense gradient. tables: [(parameter, touched row ids)]."""
    if world <= 1:
        return
    for p, rows in tables:
        if p.grad is None:
            continue
        g = p.grad
        rows = (torch.zeros(0, dtype=torch.int64, device=g.device) if rows is None
                else rows.to(torch.int64))
        vals = g[rows]
        cnt = torch.tensor([rows.numel()], dtype=torch.int64, device=g.device)
        cnts = torch.empty(world, dtype=torch.int64, device=g.device)
        dist.all_gather_into_tensor(cnts, cnt, group=group)
        cnts = cnts.tolist()
        m = max(cnts)
        if m == 0:
            continue
        r_pad = torch.zeros(m, dtype=torch.int64, device=g.device)
        v_pad = torch.zeros(m, g.shape[1], dtype=g.dtype, device=g.device)
        r_pad[:rows.numel()] = rows
        v_pad[:rows.numel()] = vals
        r_all = torch.empty(world * m, dtype=torch.int64, device=g.device)
        v_all = torch.empty(world * m, g.shape[1], dtype=g.dtype, device=g.device)
        dist.all_gather_into_tensor(r_all, r_pad, group=group)
        dist.all_gather_into_tensor(v_all, v_pad, group=group)
        g.index_fill_(0, rows, 0.0)
        for r in range(world):                   # rank order: identical sums on every rank
            rr = r_all[r * m:r * m + cnts[r]]
            g.index_add_(0, rr, v_all[r * m:r * m + cnts[r]])
        touched = torch.unique(torch.cat([r_all[r * m:r * m + cnts[r]] for r in range(world)]))
        g[touched] /= world


def train_step(model, opt, batch, x_dict, edge_type, node_type, local_node_idx, y_global, world):
    """mag/regnn_ns.py:399-407 with the gradient all-reduce between backward and step (dense
    parameters in one flat bucket; feats_type-2 embedding tables by touched rows)."""
    batch_size, n_id, adjs = batch
    opt.zero_grad(set_to_none=True)
    out = model(n_id, x_dict, adjs, edge_type, node_type, local_node_idx)
    y = y_global[n_id][:batch_size].squeeze(-1)
    loss = F.nll_loss(out, y)
    loss.backward()
    tables = model.embedding_tables() if hasattr(model, "embedding_tables") else []
    table_ids = {id(p) for p, _ in tables}
    flat_grad_allreduce([p for p in model.parameters() if id(p) not in table_ids], world)
    sparse_rows_allreduce(tables, world)
    opt.step()
    return loss
