"""Layer-wise full-neighbour inference of the neighbour-sampled REGNN (mag/regnn_ns.py:348-369),
sharded over data-parallel ranks by destination rows.

The reference walks ``subgraph_loader`` (PyG NeighborSampler, sizes=[-1], node_idx=None) batch by
batch with ``x_all`` on the host and a host<->device copy per batch. A batch with every in-edge is
just a row range of the full graph, so here each layer is ONE full-graph mean aggregation per
rank over the rank's own destination rows, with the layer input resident in HBM:

    rank r owns rows [b_r, b_{r+1})      (boundaries balance in-edges + rows)
    xs_r   = x_r @ W_l                    (mag/regnn_layers.py:101-102, own rows only)
    xs     = all_gather(xs_r)             (RCCL over xGMI; one exchange per layer)
    out_r  = mean_{e: u->v} ew_e xs[u] + bias  (+ xs_r if residual), LayerNorm, relu
                                          (mag/regnn_layers.py:110-150, regnn_ns.py:361-362)

Exchanging the projected rows (xs) instead of the layer input (x) lets every rank project only
the rows it owns. The aggregation is the same HIP SpMM as training (relation table, 1/in-count
and bias fused; hub rows through the chunk + tree path). Each block holds the rank's CSR row
range with the target self loops appended last in every row, as the sampled blocks do
(mag/regnn_layers.py:90-96), so a rank's output rows equal the reference's batch outputs.
"""
import torch
import torch.distributed as dist
import torch.nn.functional as F

from . import ops
from .graph import SegPlan, _word_padded


def shard_bounds(csr_ptr, world):
    """row boundaries [b_0=0, ..., b_W=N] that balance (in-edges + rows) across ranks."""
    n = csr_ptr.numel() - 1
    if world <= 1:
        return [0, n]
    cost = csr_ptr.to(torch.int64) + torch.arange(n + 1, device=csr_ptr.device)
    total = int(cost[-1].item())
    want = torch.tensor([total * r // world for r in range(1, world)], dtype=torch.int64,
                        device=csr_ptr.device)
    cut = torch.searchsorted(cost, want).tolist()
    b = [0] + [min(max(int(c), 0), n) for c in cut] + [n]
    for i in range(1, len(b)):
        b[i] = max(b[i], b[i - 1])
    return b


class RowBlock:
    """Forward-only CSR of destination rows [r0, r1) of a global graph (all N nodes as sources),
    a self loop appended last in every row with relation type ntype + num_edge_types.

    Exposes what ops.re_spmm's forward reads (RelGraph-compatible: csr_ptr / csr_idx / csr_plan /
    n_src / n_dst / E, and pack.rel_csr with 0-based relation ids)."""

    def __init__(self, rg, r0, r1, edge_type_csr, node_type, num_edge_types):
        dev = rg.device
        ptr = rg.csr_ptr.to(torch.int64)
        e0, e1 = int(ptr[r0].item()), int(ptr[r1].item())
        n = r1 - r0
        M = e1 - e0
        cnt = ptr[r0 + 1:r1 + 1] - ptr[r0:r1]
        newptr = torch.zeros(n + 1, dtype=torch.int64, device=dev)
        torch.cumsum(cnt + 1, 0, out=newptr[1:])
        row_of = torch.repeat_interleave(torch.arange(n, device=dev), cnt, output_size=M)
        posn = torch.arange(M, device=dev) + row_of          # row i's edges shift by i loops
        loop_pos = newptr[1:] - 1
        idx = torch.empty(M + n, dtype=torch.int32, device=dev)
        idx[posn] = rg.csr_idx[e0:e1]
        idx[loop_pos] = torch.arange(r0, r1, dtype=torch.int32, device=dev)
        rel = torch.empty(M + n, dtype=torch.uint8, device=dev)
        rel[posn] = edge_type_csr[e0:e1]
        rel[loop_pos] = (node_type[r0:r1] + num_edge_types).to(torch.uint8)
        del posn, row_of
        self.device, self.r0, self.r1 = dev, r0, r1
        self.n_src, self.n_dst, self.E = rg.n_src, n, M + n
        self.csr_ptr = newptr.to(torch.int32).contiguous()
        self.csr_idx = idx
        self.csr_plan = SegPlan(self.csr_ptr)
        self.pack = type("RowPack", (), {})()
        self.pack.rel_csr = _word_padded(rel)
        self._inv = (1.0 / (cnt + 1).to(torch.float32)).contiguous()   # mean over edges + loop

    def inv_in_count(self):
        return self._inv


def exchange_rows(x_loc, bounds, rank, world, group=None):
    """all-gather of every rank's row block into the full [N, F] tensor (uneven row counts are
    padded to the largest shard for one all_gather_into_tensor call)."""
    if world <= 1:
        return x_loc
    rows = [bounds[r + 1] - bounds[r] for r in range(world)]
    m = max(rows)
    Fw = x_loc.shape[1]
    send = x_loc
    if x_loc.shape[0] != m:
        send = torch.zeros(m, Fw, dtype=x_loc.dtype, device=x_loc.device)
        send[:x_loc.shape[0]] = x_loc
    buf = torch.empty(world * m, Fw, dtype=x_loc.dtype, device=x_loc.device)
    dist.all_gather_into_tensor(buf, send.contiguous(), group=group)
    if all(r == m for r in rows):
        return buf
    return torch.cat([buf[r * m:r * m + rows[r]] for r in range(world)], 0)


class ShardedInference:
    """The rank-local half of REGNN.inference: holds this rank's RowBlock and steps the layers.

    run() drives the per-layer exchange through torch.distributed; the step methods let a caller
    (tests) drive several ranks in lockstep within one process."""

    def __init__(self, model, rg, edge_type, node_type, local_node_idx, rank=0, world=1,
                 bounds=None):
        if getattr(model, "model", "regcn") != "regcn":
            raise NotImplementedError("sharded full-neighbour inference covers the REGCN model")
        if model.self_loop_type != 2:
            raise NotImplementedError("full-neighbour inference is built for self_loop_type=2 "
                                      "(the mag/regnn_ns.py default)")
        self.model, self.rank, self.world = model, rank, world
        self.node_type, self.local_node_idx = node_type, local_node_idx
        self.bounds = bounds if bounds is not None else shard_bounds(rg.csr_ptr, world)
        r0, r1 = self.bounds[rank], self.bounds[rank + 1]
        self.r0, self.r1 = r0, r1
        et_csr = edge_type.to(rg.device)[rg.csr_eid].to(torch.uint8)
        self.block = RowBlock(rg, r0, r1, et_csr, node_type, model.num_edge_types)
        self.own = torch.arange(r0, r1, device=rg.device)

    @torch.no_grad()
    def project(self, layer, x_loc):
        return x_loc @ self.model.convs[layer].weight                      # :101-102

    @torch.no_grad()
    def input(self, x_dict, layer=0):
        """group_input for the own rows (mag/regnn_ns.py:300-326). Node ids are type-contiguous
        (the mag node numbering), so each type's Linear is one GEMM over its row range written
        in place; otherwise the model's generic group_input."""
        m = self.model
        nt = self.node_type[self.r0:self.r1]
        x = None
        if nt.numel() and bool((nt[1:] >= nt[:-1]).all()):
            x = torch.empty(nt.numel(), m.hidden_dim, device=nt.device)
            types = torch.unique_consecutive(nt).tolist()
            bounds = torch.searchsorted(nt, torch.tensor(types + [types[-1] + 1],
                                                         device=nt.device)).tolist()
            loc = self.local_node_idx[self.r0:self.r1]
            for k, t in enumerate(types):
                a, b = bounds[k], bounds[k + 1]
                l0 = int(loc[a].item())
                xt = x_dict[t]
                lin = m.lins[str(t)]
                ar = torch.arange(l0, l0 + (b - a), device=loc.device)
                if bool((loc[a:b] == ar).all()):                  # contiguous local ids
                    torch.addmm(lin.bias, xt[l0:l0 + (b - a)], lin.weight.t(), out=x[a:b])
                else:
                    torch.addmm(lin.bias, xt[loc[a:b]], lin.weight.t(), out=x[a:b])
        if x is None:
            x = m.group_input(x_dict, self.node_type, self.local_node_idx, self.own)
        return x, self.project(layer, x)

    @torch.no_grad()
    def aggregate(self, layer, xs_all, xs_loc):
        """one HIP pass: mean aggregation with the relation table and bias, + residual,
        LayerNorm and relu fused in the epilogue (regnn_spmm_fwd_fused)."""
        conv = self.model.convs[layer]
        tab = F.leaky_relu(conv.relation_weight * conv.scaling_factor)     # :110-111
        blk = self.block
        res = xs_loc if conv.residual else None                            # x_target @ W
        if conv.use_norm == 'bn':
            out = ops.re_spmm(blk, xs_all, tab, blk.pack, post=blk.inv_in_count(),
                              bias=conv.bias)
            out = F.relu(conv.norm(out + res if res is not None else out))
            return out
        ln = None
        if conv.use_norm == 'ln':
            ln = (conv.norm.weight, conv.norm.bias, conv.norm.eps)
        return ops.re_spmm_fused(blk, xs_all, tab, blk.pack, post=blk.inv_in_count(),
                                 bias=conv.bias, residual=res, ln=ln, relu=True)

    @torch.no_grad()
    def head(self, x_loc):
        return self.model.out_lin(x_loc)                                   # :367

    @torch.no_grad()
    def head_argmax(self, x_loc):
        lin = self.model.out_lin
        return ops.head_argmax(x_loc, lin.weight, lin.bias)

    @torch.no_grad()
    def run(self, x_dict, gather="logits", group=None):
        """-> this rank's logits rows [r0, r1) (gather=None), or every row all-gathered
        (gather='logits'), or the all-gathered argmax (gather='argmax', int64 [N])."""
        L = self.model.num_layers
        _, xs = self.input(x_dict, 0)
        for layer in range(L):
            xs_all = exchange_rows(xs, self.bounds, self.rank, self.world, group)
            x = self.aggregate(layer, xs_all, xs)
            del xs_all
            if layer + 1 < L:
                xs = self.project(layer + 1, x)
        if gather == "argmax":
            am = self.head_argmax(x)
            return exchange_rows(am.unsqueeze(1), self.bounds, self.rank, self.world,
                                 group).squeeze(1)
        logits = self.head(x)
        if gather is None:
            return logits
        return exchange_rows(logits, self.bounds, self.rank, self.world, group)
