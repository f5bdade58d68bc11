"""Device-resident neighbour-sampled (NS) step for the ogbn-mag path (mag/regnn_ns.py:206-214,
392-420) on MI355X: sampler, block aggregation, model step and optimizer with no host
synchronisation, so one training step is one HIP-graph replay.

* ``DeviceSampler`` — the per-hop sampler (regnn_ns_hop, include/regnn_hip.h) over buffers sized
  by capacity: batch B, then B*(k0+1), B*(k0+1)*(k1+1), ... targets / sources per hop. Counts live
  on the device (``sizes``); every later kernel reads them there.
* ``NSBlock`` — one hop's sampled block in the layout its aggregation reads (CSR by target,
  local ids, self loop last, uint8 relation ids, 1/in-count); RelGraph-compatible for ops.
* ``NSTrainer`` — one rank's data-parallel NS training step (regnn_ns_batch -> hops -> REGNN
  forward / nll / backward -> flat-bucket all-reduce -> Adam), captured in a HIP graph when
  asked. Rank r of W takes global batches r, r+W, ... of the epoch's shared permutation
  (SURVEY.md §8e); every rank runs the same number of steps per epoch.

The sampled indices follow the build's sampler spec (oracle/sampler_oracle.py, bit-exact).
"""
import torch
import torch.nn.functional as F

from . import _lib as L

M64 = (1 << 64) - 1


def _i64(u):
    """an unsigned 64-bit value as the int64 with the same bits."""
    u &= M64
    return u - (1 << 64) if u >= (1 << 63) else u


class NSBlock:
    """A sampled bipartite block (sources = n_id[:n_src], targets = n_id[:n_dst]).

    csr_ptr [n_dst+1] int32, csr_idx [E] local source ids (row v's self loop last), rel [E]
    uint8 0-based relation (edge type; num_edge_types + node type for the loop), pos [E] CSR
    position of the sampled edge in the global graph (-1: loop), inv [n_dst] 1/(sampled + 1).
    n_dst / n_src / E are host ints: exact sizes (API path) or capacities (device engine)."""

    is_ns_block = True

    def __init__(self, ptr, idx, rel, pos, inv, n_dst, n_src, E, device):
        self.csr_ptr, self.csr_idx, self.rel, self.pos, self.inv = ptr, idx, rel, pos, inv
        self.n_dst, self.n_src, self.E = int(n_dst), int(n_src), int(E)
        self.device = device

    def __iter__(self):                     # (edge_index, e_id, size) unpacking of the reference
        return iter((self, None, (self.n_src, self.n_dst)))

    def to(self, device):
        return self


class DeviceSampler:
    """Capacity-sized device sampler over a RelGraph (CSR by destination).

    etype: 0-based edge type per caller edge (mag edge_type), or None (relation 0);
    ntype: node type per global node (self-loop relation num_edge_types + ntype), or None."""

    def __init__(self, rg, sizes, batch_size, etype=None, ntype=None, num_edge_types=0):
        dev = rg.device
        self.rg, self.device = rg, dev
        self.sizes_k = [int(k) for k in sizes]
        if not self.sizes_k or any(k < 1 or k > 64 for k in self.sizes_k):
            raise ValueError(f"device sampler fan-outs must lie in [1, 64], got {sizes}")
        if len(self.sizes_k) > 6:
            raise ValueError("at most 6 hops")
        self.B = int(batch_size)
        caps = [self.B]
        for k in self.sizes_k:
            caps.append(caps[-1] * (k + 1))
        if caps[-1] >= 2 ** 31:
            raise ValueError(f"sampler capacity {caps[-1]} exceeds int32")
        self.caps = caps
        self.num_edge_types = int(num_edge_types)
        n_nodes = max(rg.n_src, rg.n_dst)
        if etype is None:
            self.etype_csr = torch.zeros(rg.E, dtype=torch.uint8, device=dev)
        else:
            et = torch.as_tensor(etype).to(dev).reshape(-1)
            if et.numel() != rg.E:
                raise ValueError(f"etype has {et.numel()} entries, graph has {rg.E} edges")
            self.etype_csr = et[rg.csr_eid].to(torch.uint8).contiguous()
        if ntype is None:
            self.ntype = torch.zeros(n_nodes, dtype=torch.int32, device=dev)
        else:
            self.ntype = torch.as_tensor(ntype).to(dev).to(torch.int32).contiguous()
        if int(self.num_edge_types) + (int(self.ntype.max().item()) if self.ntype.numel() else 0) > 255:
            raise ValueError("relation ids must fit uint8")
        self.state = torch.zeros(8, dtype=torch.int64, device=dev)
        self.sizes = torch.zeros(16, dtype=torch.int32, device=dev)
        self.n_id = torch.zeros(caps[-1], dtype=torch.int32, device=dev)
        self.g2l = torch.zeros(n_nodes, dtype=torch.int64, device=dev)
        self.first = torch.full((n_nodes,), -1, dtype=torch.int64, device=dev)
        self.hop_bufs, self.blocks = [], []
        for h, k in enumerate(self.sizes_k):
            cd = caps[h]
            ce = cd * (k + 1)
            nt = (ce + 1023) // 1024
            z = lambda n, dt=torch.int32: torch.zeros(n, dtype=dt, device=dev)  # noqa: E731
            self.hop_bufs.append(dict(samp=z(cd * k), spos=z(cd * k), scnt=z(cd), gsrc=z(ce),
                                      flag=z(ce, torch.uint8), tiles=z(nt + 1)))
            blk = NSBlock(z(cd + 1), z(ce), z(ce, torch.uint8), z(ce),
                          torch.ones(cd, dtype=torch.float32, device=dev), cd, caps[h + 1], ce, dev)
            self.blocks.append(blk)

    # -- the per-step device work ------------------------------------------------------------
    def batch_from_perm(self, perm, rank=0, world=1):
        """regnn_ns_batch: this rank's next targets from the epoch permutation (device int64)."""
        L.call("regnn_ns_batch", L.ptr(perm), perm.numel(), self.B, int(rank), int(world),
               L.ptr(self.state), L.ptr(self.n_id), L.ptr(self.sizes), L.stream())

    def run_hops(self):
        rg = self.rg
        for h, k in enumerate(self.sizes_k):
            b, blk = self.hop_bufs[h], self.blocks[h]
            L.call("regnn_ns_hop", L.ptr(rg.csr_ptr), L.ptr(rg.csr_idx), L.ptr(self.etype_csr),
                   L.ptr(self.ntype), self.num_edge_types, k, h, L.ptr(self.state),
                   L.ptr(self.sizes), L.ptr(self.n_id), self.caps[h], L.ptr(self.g2l),
                   L.ptr(self.first), L.ptr(b["samp"]), L.ptr(b["spos"]), L.ptr(b["scnt"]),
                   L.ptr(b["gsrc"]), L.ptr(b["flag"]), L.ptr(b["tiles"]), L.ptr(blk.csr_ptr),
                   L.ptr(blk.csr_idx), L.ptr(blk.rel), L.ptr(blk.pos), L.ptr(blk.inv),
                   L.stream())

    def set_seed(self, base_seed, epoch, batch_idx):
        """host-driven batches (the PyG-style iterator): seed words + a fresh dedup stamp."""
        st = self.state.cpu()
        st[0], st[1], st[3] = _i64(int(base_seed)), int(epoch), int(batch_idx)
        st[4] += 1
        self.state.copy_(st)

    def set_targets(self, targets):
        n = int(targets.numel())
        if n > self.B:
            raise ValueError(f"{n} targets exceed the sampler's batch capacity {self.B}")
        self.n_id[:n].copy_(targets.to(torch.int32))
        self.sizes[0:1].fill_(n)

    def model_blocks(self):
        """blocks in the model's layer order (outermost hop first, PyG adjs[::-1])."""
        return self.blocks[::-1]

    def exact_adjs(self):
        """PyG-style per-hop output at exact sizes (one host sync): [(edge_index [2, M] local
        (src, dst) without self loops, dst-major; e_id; (n_src, n_dst); NSBlock copy)], hop
        order (innermost first)."""
        sz = self.sizes.cpu().tolist()
        out = []
        for h in range(len(self.sizes_k)):
            blk = self.blocks[h]
            n_dst, n_src, E = sz[h], sz[h + 1], sz[8 + h]
            ptr = blk.csr_ptr[:n_dst + 1].clone()
            idx, rel, pos = blk.csr_idx[:E].clone(), blk.rel[:E].clone(), blk.pos[:E].clone()
            inv = blk.inv[:n_dst].clone()
            cnt = (ptr[1:] - ptr[:-1]).to(torch.int64)
            dst_all = torch.repeat_interleave(torch.arange(n_dst, device=self.device), cnt)
            keep = pos >= 0
            src_l = idx[keep].to(torch.int64)
            dst_l = dst_all[keep]
            e_id = self.rg.csr_eid[pos[keep].to(torch.int64)]
            eb = NSBlock(ptr, idx, rel, pos, inv, n_dst, n_src, E, self.device)
            out.append((torch.stack([src_l, dst_l]), e_id, (n_src, n_dst), eb, cnt - 1))
        return sz[len(self.sizes_k)], out


class NSTrainer:
    """One rank's NS training step (mag/regnn_ns.py:392-420) on the device sampler.

    model: mag.REGNN; opt: an optimizer over model.parameters() (Adam(capturable=True) for
    graph capture); train_idx: target nodes (the paper train split); y_global [N, 1] labels.
    The gradients live in one flat fp32 bucket (p.grad are views of it): one RCCL all-reduce
    per step for world > 1 (mag.flat_grad_allreduce's exchange), outside the captured graph."""

    def __init__(self, model, opt, rg, sizes, batch_size, train_idx, x_dict, edge_type,
                 node_type, local_node_idx, y_global, num_edge_types, seed=0, rank=0, world=1,
                 shuffle=True):
        self.model, self.opt = model, opt
        dev = rg.device
        self.device, self.rank, self.world = dev, int(rank), int(world)
        self.sampler = DeviceSampler(rg, sizes, batch_size, etype=edge_type, ntype=node_type,
                                     num_edge_types=num_edge_types)
        self.train_idx = torch.as_tensor(train_idx).to(dev, torch.int64)
        self.perm = self.train_idx.clone()
        self.shuffle, self.seed = shuffle, int(seed)
        self.x_dict, self.node_type, self.local_node_idx = x_dict, node_type, local_node_idx
        self.y_flat = y_global.reshape(-1).to(dev, torch.int64)
        self.params = [p for p in model.parameters() if p.requires_grad]
        n = sum(p.numel() for p in self.params)
        self.flat = torch.zeros(n, dtype=torch.float32, device=dev)
        o = 0
        for p in self.params:
            p.grad = self.flat[o:o + p.numel()].view_as(p)
            o += p.numel()
        self.loss_sum = torch.zeros((), dtype=torch.float32, device=dev)
        self.loss = torch.zeros((), dtype=torch.float32, device=dev)
        self.graphs = None
        self.epoch = -1
        self.set_epoch(0)

    # -- epochs ----------------------------------------------------------------------------------
    def steps_per_epoch(self):
        nb = -(-self.train_idx.numel() // self.sampler.B)
        return -(-nb // self.world)

    def set_epoch(self, epoch):
        """shared per-epoch permutation (every rank draws the same one: NeighborSampler's order)."""
        self.epoch = int(epoch)
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed * 1_000_003 + self.epoch)
            order = torch.randperm(self.train_idx.numel(), generator=g).to(self.device)
            self.perm.copy_(self.train_idx[order])
        else:
            self.perm.copy_(self.train_idx)
        st = self.sampler.state
        st[0:1].fill_(_i64(self.seed))
        st[1:2].fill_(self.epoch)
        st[2:3].zero_()

    # -- one step --------------------------------------------------------------------------------
    def _forward_backward(self):
        s = self.sampler
        self.flat.zero_()
        s.batch_from_perm(self.perm, self.rank, self.world)
        s.run_hops()
        B = s.B
        n_id = s.n_id.to(torch.int64)
        out = self.model(n_id, self.x_dict, s.model_blocks(), None, self.node_type,
                         self.local_node_idx)
        y = self.y_flat[n_id[:B]]
        valid = torch.arange(B, device=self.device) < s.sizes[0]
        y = torch.where(valid, y, torch.full_like(y, -100))
        loss = F.nll_loss(out, y)                     # mean over the batch's targets
        loss.backward()
        with torch.no_grad():
            self.loss.copy_(loss.detach())
            self.loss_sum.add_(loss.detach() * s.sizes[0].to(torch.float32))

    def _exchange(self):
        if self.world > 1:
            import torch.distributed as dist
            dist.all_reduce(self.flat, op=dist.ReduceOp.SUM)
            self.flat.div_(self.world)

    def step(self):
        """one eager step (host-launched; no host synchronisation)."""
        self._forward_backward()
        self._exchange()
        self.opt.step()

    def capture(self, warmup=2):
        """capture the step as HIP graphs: [fwd/bwd] (+ the eager all-reduce) + [optimizer]."""
        side = torch.cuda.Stream(device=self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        st0 = self.sampler.state.clone()
        with torch.cuda.stream(side):
            for _ in range(warmup):
                self.step()
        torch.cuda.current_stream(self.device).wait_stream(side)
        torch.cuda.synchronize(self.device)
        # warm-up steps do not advance the epoch (batch counter, edge counter); the dedup stamp
        # (state[4]) stays monotone: the tables still hold the warm-up steps' stamps
        st = self.sampler.state
        st[2:4].copy_(st0[2:4])
        st[5:6].copy_(st0[5:6])
        g1 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g1):
            self._forward_backward()
        g2 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g2):
            self.opt.step()
        self.graphs = (g1, g2)

    def replay(self):
        g1, g2 = self.graphs
        g1.replay()
        self._exchange()
        g2.replay()

    def edges_total(self):
        """aggregated edges of every step so far (device counter: one host sync)."""
        return int(self.sampler.state[5].item())
