"""GPU neighbour sampler with PyG ``NeighborSampler``'s iteration contract (mag/regnn_ns.py:206-214,
consumed at :399-401 and :337-341), sharded over data-parallel ranks.

Each hop: regnn_sample_count -> prefix sum -> regnn_sample_fill (one wave per target, Floyd
sampling, spec in include/regnn_hip.h) -> first-seen de-duplication of the new source nodes with
device tensor ops (amin-scatter of candidate positions: order independent, so deterministic).
Output is bit-identical to oracle/sampler_oracle.py for the same seeds.
"""
import torch

from . import _lib as L

M64 = (1 << 64) - 1


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
    e_id = original edge ids, size = (n_src, n_dst); ``rel`` = 0-based relation of every edge."""

    def __init__(self, edge_index, e_id, size, csr_pos, counts=None):
        self.edge_index, self.e_id, self.size, self.csr_pos = edge_index, e_id, size, csr_pos
        self.counts = counts       # sampled in-edges per target (int32), dst-major order

    def __iter__(self):
        return iter((self.edge_index, self.e_id, self.size))

    def to(self, device):
        return self


class NeighborSampler:
    """Iterates (batch_size, n_id, adjs) over shuffled target batches; rank r of W takes global
    batches r, r+W, ... of a shared per-epoch permutation."""

    def __init__(self, rg, node_idx, sizes, batch_size, shuffle=True, seed=0, rank=0,
                 world_size=1, drop_last=False):
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
        n = rg.n_dst
        self._g2l = torch.full((n,), -1, dtype=torch.int64, device=rg.device)
        self._first = torch.full((n,), 1 << 62, dtype=torch.int64, device=rg.device)

    def set_epoch(self, epoch):
        self.epoch = int(epoch)

    def _order(self):
        if not self.shuffle:
            return self.node_idx
        g = torch.Generator()
        g.manual_seed(self.seed * 1_000_003 + self.epoch)
        perm = torch.randperm(self.node_idx.numel(), generator=g)
        return self.node_idx[perm.to(self.node_idx.device)]

    def num_batches(self):
        n = self.node_idx.numel()
        nb = n // self.batch_size if self.drop_last else -(-n // self.batch_size)
        return len(range(self.rank, nb, self.world))

    def __len__(self):
        return self.num_batches()

    def batches(self):
        """(global batch index, target nodes) of this rank for the current epoch."""
        order = self._order()
        n = order.numel()
        nb = n // self.batch_size if self.drop_last else -(-n // self.batch_size)
        for b in range(self.rank, nb, self.world):
            yield b, order[b * self.batch_size:(b + 1) * self.batch_size]

    def __iter__(self):
        for b, batch in self.batches():
            yield self.sample(batch, b)

    def sample(self, batch, batch_idx=0):
        n_id = batch.to(self.rg.device, torch.int64)
        adjs = []
        for hop, k in enumerate(self.sizes):
            seed = hop_seed(self.seed, self.epoch, batch_idx, hop)
            n_dst = n_id.numel()
            n_id, src_l, dst_l, pos, counts = self.sample_hop(n_id, k, seed)
            e_id = self.rg.csr_eid[pos]
            adjs.append(Adj(torch.stack([src_l, dst_l]), e_id, (n_id.numel(), n_dst), pos, counts))
        return batch.numel(), n_id, adjs[0] if len(adjs) == 1 else adjs[::-1]

    def sample_hop(self, targets, k, seed):
        rg, dev = self.rg, self.rg.device
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
