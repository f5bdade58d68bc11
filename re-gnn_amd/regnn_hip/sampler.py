"""GPU neighbour sampler with PyG ``NeighborSampler``'s iteration contract (mag/regnn_ns.py:206-214,
consumed at :399-401 and :337-341), sharded over data-parallel ranks.

Fan-outs in [1, 64] run on the device sampler (regnn_hip.ns.DeviceSampler: regnn_ns_hop, no host
sizes; the only host synchronisation is reading the exact sizes once per batch for the PyG-style
Adj objects). A fan-out of -1 (all neighbours, the reference's subgraph_loader) or above 64 takes
the count / prefix-sum / fill path with device first-seen de-duplication. Both follow the same
spec and are bit-identical to oracle/sampler_oracle.py for the same seeds.
"""
import torch

from . import _lib as L
from .ns import M64, DeviceSampler, NSBlock  # noqa: F401  (NSBlock re-exported)


def _mix(x):
    x &= M64
    x ^= x >> 30
    x = (x * 0xBF58476D1CE4E5B9) & M64
    x ^= x >> 27
    x = (x * 0x94D049BB133111EB) & M64
    x ^= x >> 31
    return x


def hop_seed(base, epoch, batch, hop):
    """per-(epoch, batch, hop) 64-bit sampler seed (spec shared with the oracle)."""
    return _mix((base & M64) ^ _mix((epoch << 40) ^ (batch << 8) ^ hop))


class Adj:
    """One sampled block, PyG ``EdgeIndex``-compatible: (edge_index, e_id, size) unpacking.

    edge_index = [src_local, dst_local] (dst-major: rows already grouped by target),
    e_id = original edge ids, size = (n_src, n_dst); ``block`` = the same block in the layout
    the aggregation reads (regnn_hip.ns.NSBlock; relation ids filled from the sampler's edge
    types when it has them, else by the model from edge_type[e_id])."""

    def __init__(self, edge_index, e_id, size, counts=None, block=None):
        self.edge_index, self.e_id, self.size = edge_index, e_id, size
        self.counts = counts       # sampled in-edges per target (int64), dst-major order
        self.block = block

    def __iter__(self):
        return iter((self.edge_index, self.e_id, self.size))

    def to(self, device):
        return self


class NeighborSampler:
    """Iterates (batch_size, n_id, adjs) over shuffled target batches; rank r of W takes global
    batches r, r+W, ... of a shared per-epoch permutation. Every rank yields the
    same number of batches, ceil(nb / W): a rank past the last global batch wraps to the first
    ones (as DistributedSampler pads), so a per-step gradient all-reduce never waits on a rank
    that has finished its epoch.

    edge_type / node_type / num_edge_types (optional): the blocks' relation ids are then formed
    by the sampler itself (mag self_loop_type 2: edge type, num_edge_types + node type for the
    target's self loop)."""

    def __init__(self, rg, node_idx, sizes, batch_size, shuffle=True, seed=0, rank=0,
                 world_size=1, drop_last=False, edge_type=None, node_type=None,
                 num_edge_types=0):
        self.rg = rg
        if node_idx is None:                       # PyG: every node is a target
            node_idx = torch.arange(rg.n_dst, device=rg.device)
        self.node_idx = torch.as_tensor(node_idx).to(rg.device, torch.int64)
        self.sizes = list(sizes)
        self.batch_size = int(batch_size)
        self.shuffle, self.seed = shuffle, int(seed)
        self.rank, self.world = rank, world_size
        self.drop_last = drop_last
        self.epoch = 0
        self.edge_type, self.node_type = edge_type, node_type
        self.num_edge_types = int(num_edge_types)
        self.typed = edge_type is not None and node_type is not None
        self._dev = None
        self._g2l = self._first = None

    def set_epoch(self, epoch):
        self.epoch = int(epoch)

    def _order(self):
        if not self.shuffle:
            return self.node_idx
        g = torch.Generator()
        g.manual_seed(self.seed * 1_000_003 + self.epoch)
        perm = torch.randperm(self.node_idx.numel(), generator=g)
        return self.node_idx[perm.to(self.node_idx.device)]

    def _global_batches(self):
        n = self.node_idx.numel()
        return n // self.batch_size if self.drop_last else -(-n // self.batch_size)

    def num_batches(self):
        nb = self._global_batches()
        return -(-nb // self.world) if nb else 0

    def __len__(self):
        return self.num_batches()

    def batches(self):
        """(global batch index, target nodes) of this rank for the current epoch."""
        order = self._order()
        nb = self._global_batches()
        for j in range(self.num_batches()):
            b = (self.rank + j * self.world) % nb
            yield b, order[b * self.batch_size:(b + 1) * self.batch_size]

    def __iter__(self):
        for b, batch in self.batches():
            yield self.sample(batch, b)

    def _device_sampler(self):
        if self._dev is None:
            self._dev = DeviceSampler(
                self.rg, self.sizes, self.batch_size,
                etype=self.edge_type if self.typed else None,
                ntype=self.node_type if self.typed else None,
                num_edge_types=self.num_edge_types)
        return self._dev

    def sample(self, batch, batch_idx=0):
        if all(1 <= k <= 64 for k in self.sizes):
            ds = self._device_sampler()
            ds.set_seed(self.seed, self.epoch, batch_idx)
            ds.set_targets(batch.to(self.rg.device))
            ds.run_hops()
            n_total, hops = ds.exact_adjs()
            adjs = [Adj(ei, e_id, size, cnt, blk if self.typed else None)
                    for ei, e_id, size, blk, cnt in hops]
            n_id = ds.n_id[:n_total].to(torch.int64)
            return batch.numel(), n_id, adjs[0] if len(adjs) == 1 else adjs[::-1]
        n_id = batch.to(self.rg.device, torch.int64)
        adjs = []
        for hop, k in enumerate(self.sizes):
            seed = hop_seed(self.seed, self.epoch, batch_idx, hop)
            n_dst = n_id.numel()
            n_id, src_l, dst_l, pos, counts = self.sample_hop(n_id, k, seed)
            e_id = self.rg.csr_eid[pos]
            adjs.append(Adj(torch.stack([src_l, dst_l]), e_id, (n_id.numel(), n_dst),
                            counts.to(torch.int64)))
        return batch.numel(), n_id, adjs[0] if len(adjs) == 1 else adjs[::-1]

    def sample_hop(self, targets, k, seed):
        """one hop of any fan-out (k < 0: all in-edges) with host-sized buffers."""
        rg, dev = self.rg, self.rg.device
        if self._g2l is None:
            n = max(rg.n_src, rg.n_dst)            # sources and targets share the id space
            self._g2l = torch.full((n,), -1, dtype=torch.int64, device=dev)
            self._first = torch.full((n,), 1 << 62, dtype=torch.int64, device=dev)
        n = targets.numel()
        t32 = targets.to(torch.int32).contiguous()
        counts = torch.empty(n, dtype=torch.int32, device=dev)
        L.call("regnn_sample_count", L.ptr(rg.csr_ptr), L.ptr(t32), n, int(k), L.ptr(counts),
               L.stream())
        offs = torch.zeros(n + 1, dtype=torch.int32, device=dev)
        torch.cumsum(counts, 0, out=offs[1:])
        M = int(offs[-1].item())
        src = torch.empty(M, dtype=torch.int32, device=dev)
        pos = torch.empty(M, dtype=torch.int32, device=dev)
        L.call("regnn_sample_fill", L.ptr(rg.csr_ptr), L.ptr(rg.csr_idx), L.ptr(t32), n, int(k),
               seed & M64, L.ptr(offs), L.ptr(src), L.ptr(pos), L.stream())
        dst_l = torch.repeat_interleave(torch.arange(n, device=dev), counts.to(torch.int64))
        cand = src.to(torch.int64)
        g2l, first = self._g2l, self._first
        g2l[targets] = torch.arange(n, device=dev)
        is_new = g2l[cand] < 0
        p = torch.arange(M, device=dev)
        first.scatter_reduce_(0, cand[is_new], p[is_new], "amin")
        firstflag = is_new & (first[cand] == p)
        new_nodes = cand[firstflag]
        g2l[new_nodes] = torch.arange(n, n + new_nodes.numel(), device=dev)
        src_l = g2l[cand]
        n_id = torch.cat([targets, new_nodes])
        g2l[n_id] = -1
        first[cand] = 1 << 62
        return n_id, src_l, dst_l, pos.to(torch.int64), counts
