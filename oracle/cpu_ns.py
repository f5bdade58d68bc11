"""CPU BASELINE for the neighbour-sampled training step (test / bench infrastructure only: imported
by tests/ and bench.py's cpu_baseline leg, never by the product path).

The reference's NS step (mag/regnn_ns.py:392-420) on the host cores, restated in PyTorch CPU ops
the way the reference composes them (PyG / torch_scatter / torch_sparse are absent here and
the reference's code does not travel, so this is the "port" baseline):

* the sampler: this build's sampler spec (oracle/sampler_oracle.py, the spec the GPU sampler is
  bit-exact against) vectorised in numpy: Floyd sampling of k in-edge positions per target,
  ascending, then first-seen de-duplication of the new sources (torch_sparse sample_adj's n_id
  contract, mag/regnn_ns.py:206-214);
* the model: REGNN (mag/regnn_ns.py:216-346) for 'regcn', self_loop_type 2, LayerNorm:
  group_input with one boolean mask and one Linear per node type (:316-324); per layer
  REGCNConv.forward (mag/regnn_layers.py:80-150): self loops appended with type ntype + 7,
  the one-hot e_feat [E, 11] @ LeakyReLU(alpha * relation_weight), x_src @ W over every sampled
  source row, the (dead) weighted degree, mean aggregation of ew * x_j (torch_scatter's mean:
  index_add + in-count), + bias, LayerNorm; relu, dropout; out_lin, log_softmax (:344-346);
* nll_loss, backward (autograd), torch.optim.Adam (mag/regnn_ns.py:404-407, :495).

Pinned in tests/test_cpu_baseline.py: the sampler bit-exact against sampler_oracle, the model's
loss and every gradient against the reference REGNN's golden vectors (mag_regnn_schema).
"""
import time

import numpy as np
import torch
import torch.nn.functional as F

M64 = np.uint64((1 << 64) - 1)


def _mix(x):
    x = x ^ (x >> np.uint64(30))
    x = x * np.uint64(0xBF58476D1CE4E5B9)
    x = x ^ (x >> np.uint64(27))
    x = x * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def _hash(seed, t, j):
    """sampler_oracle.sample_hash over arrays (uint64 arithmetic wraps mod 2^64)."""
    x = (np.uint64(seed) + np.uint64(0x9E3779B97F4A7C15) * (t.astype(np.uint64) + np.uint64(1))
         + np.uint64(0xD1B54A32D192ED03) * (j.astype(np.uint64) + np.uint64(1)))
    return _mix(x) >> np.uint64(32)


def hop_seed(base, epoch, batch, hop):
    from .sampler_oracle import hop_seed as hs
    return hs(base, epoch, batch, hop)


def sample_rows(ptr, idx, targets, k, seed):
    """sampled in-edge CSR positions of every target, target-major, ascending per target
    (sampler_oracle.sample_row over all targets at once) -> (positions, counts)."""
    targets = np.asarray(targets, np.int64)
    b = ptr[targets]
    d = ptr[targets + 1] - b
    cnt = np.minimum(d, k)
    full = d <= k
    out = np.empty((targets.size, k), np.int64)
    # rows with deg <= k: every position
    ar = np.arange(k)
    out[:] = np.where(ar[None, :] < d[:, None], ar[None, :], np.iinfo(np.int64).max)
    big = np.nonzero(~full)[0]
    if big.size:
        tb, db = targets[big], d[big]
        chosen = np.empty((big.size, k), np.int64)
        with np.errstate(over="ignore"):
            for jj in range(k):                           # Floyd: j = deg - k .. deg - 1
                j = db - k + jj
                r = _hash(seed, tb, j)
                pos = ((r * (j + 1).astype(np.uint64)) >> np.uint64(32)).astype(np.int64)
                seen = (chosen[:, :jj] == pos[:, None]).any(1) if jj else np.zeros(big.size, bool)
                chosen[:, jj] = np.where(seen, j, pos)
        out[big] = np.sort(chosen, 1)
    keep = ar[None, :] < cnt[:, None]
    pos = (out + b[:, None])[keep]
    return pos, cnt


class Sampler:
    """the NS sampler over a dst-major CSR (ptr, idx); one marker array over the global ids is
    kept between batches (only the entries a batch set are reset)."""

    def __init__(self, ptr, idx, N):
        self.ptr, self.idx = np.asarray(ptr, np.int64), np.asarray(idx, np.int64)
        self.local = np.full(int(N), -1, np.int64)

    def sample(self, batch, sizes, base_seed, epoch, batch_idx):
        """-> (n_id, adjs) with adjs = [(src_local, dst_local, e_pos, (n_src, n_dst))], outermost
        hop first (sampler_oracle.neighbor_sample, bit-identical)."""
        n_id = np.asarray(batch, np.int64)
        self.local[n_id] = np.arange(n_id.size)
        adjs = []
        for hop, k in enumerate(sizes):
            seed = hop_seed(base_seed, epoch, batch_idx, hop)
            n_dst = n_id.size
            pos, cnt = sample_rows(self.ptr, self.idx, n_id, k, seed)
            src = self.idx[pos]
            dst = np.repeat(np.arange(n_dst), cnt)
            new = self.local[src] < 0
            u, first = np.unique(src[new], return_index=True)
            fresh = u[np.argsort(first, kind="stable")]
            self.local[fresh] = n_id.size + np.arange(fresh.size)
            n_id = np.concatenate([n_id, fresh])
            adjs.append((self.local[src], dst, pos, (n_id.size, n_dst)))
        self.local[n_id] = -1
        return n_id, adjs[::-1]


def _lrelu(v):
    return F.leaky_relu(v)


class REGNNCPU(torch.nn.Module):
    """REGNN 'regcn' / self_loop_type 2 / LayerNorm (mag/regnn_ns.py:216-346) on CPU ops, with
    the reference's parameter names (lins.{t}, convs.{l}.{weight, bias, relation_weight,
    norm.*}, out_lin, norm) so the golden fixtures load by name."""

    def __init__(self, in_ch, hidden, out_ch, num_layers, alpha, dropout, T, num_edge_types=7):
        super().__init__()
        self.T, self.ne, self.alpha, self.dropout = T, num_edge_types, float(alpha), dropout
        self.lins = torch.nn.ModuleDict({str(t): torch.nn.Linear(in_ch, hidden) for t in range(T)})
        self.convs = torch.nn.ModuleList()
        for _ in range(num_layers):
            c = torch.nn.Module()
            c.weight = torch.nn.Parameter(torch.empty(hidden, hidden))
            c.bias = torch.nn.Parameter(torch.zeros(hidden))
            c.relation_weight = torch.nn.Parameter(torch.full((num_edge_types + T,), 1.0 / alpha))
            c.norm = torch.nn.LayerNorm(hidden)
            torch.nn.init.xavier_uniform_(c.weight)
            self.convs.append(c)
        self.out_lin = torch.nn.Linear(hidden, out_ch)
        self.norm = torch.nn.LayerNorm(hidden)                  # declared, unused (:250)

    def group_input(self, x_dict, node_type, local_idx):        # :316-324
        h = torch.zeros(node_type.numel(), self.out_lin.in_features, dtype=self.out_lin.weight.dtype)
        for key, x in x_dict.items():
            mask = node_type == key
            h[mask] = self.lins[str(key)](x[local_idx[mask]])
        return h

    def conv(self, c, x, x_t, src, dst, etype, tgt_type):       # regnn_layers.py:80-150
        n_t = tgt_type.numel()
        loop = torch.arange(n_t)
        src = torch.cat([src, loop])
        dst = torch.cat([dst, loop])
        et = torch.cat([etype, tgt_type + self.ne])
        e_feat = torch.zeros(et.numel(), self.ne + self.T, dtype=x.dtype).scatter_(
            1, et.view(-1, 1), 1.0)
        xs = x @ c.weight
        _ = x_t @ c.weight                                      # :107 (no residual: unused)
        rw = _lrelu(c.relation_weight * self.alpha)
        ew = e_feat @ rw
        deg = torch.zeros(n_t, dtype=x.dtype).index_add_(0, dst, ew)   # :116-126 (dead norm)
        _ = deg.pow(-1.0)[dst]
        msg = ew.view(-1, 1) * xs[src]                          # message :142-144
        s = torch.zeros(n_t, xs.shape[1], dtype=x.dtype).index_add_(0, dst, msg)
        cnt = torch.zeros(n_t, dtype=x.dtype).index_add_(0, dst, torch.ones_like(ew))
        out = s / cnt.clamp(min=1).view(-1, 1) + c.bias        # aggr='mean', update() :146-148
        return c.norm(out)

    def forward(self, n_id, x_dict, adjs, edge_type, node_type, local_idx):
        x = self.group_input(x_dict, node_type[n_id], local_idx[n_id])
        nt = node_type[n_id]
        for i, (src, dst, e_id, size) in enumerate(adjs):
            x_t = x[:size[1]]
            nt = nt[:size[1]]
            x = self.conv(self.convs[i], x, x_t, src, dst, edge_type[e_id], nt)
            x = F.relu(x)
            x = F.dropout(x, p=self.dropout, training=self.training)
        return self.out_lin(x).log_softmax(dim=-1)


def step_baseline(scale=1.0, steps=10, warm=3, batch=512, sizes=(25, 20), hidden=64,
                  classes=349, threads=None):
    """time the NS training step on the host cores: mag_like(scale) (the bench's generator at
    that scale, CPU), feats_type 3 (128-d), REGNN hidden 64, dropout 0.5, Adam lr 1e-3. The graph
    build is untimed; each timed step = sampling + forward + nll + backward + Adam. Returns
    (median s/step, median aggregated edges/step incl. self loops, info)."""
    import sys
    import os
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "re-gnn_amd"))
    from regnn_hip import synth
    prev = torch.get_num_threads()
    if threads:
        torch.set_num_threads(int(threads))
    try:
        gd = synth.mag_like(scale, seed=0, device="cpu")
        keep = gd["rel"] <= 7
        src = gd["src"][keep].numpy()
        dst = gd["dst"][keep].numpy()
        et = (gd["rel"][keep].to(torch.int64) - 1)
        N = gd["N"]
        del gd["src"], gd["dst"], gd["rel"], keep
        order = np.argsort(dst, kind="stable")
        idx = src[order]
        etype_csr = et[torch.from_numpy(order)]
        ptr = np.zeros(N + 1, np.int64)
        ptr[1:] = np.cumsum(np.bincount(dst, minlength=N))
        del src, dst, order
        node_type = gd["ntype"].cpu()
        offs = torch.tensor([gd["type_offsets"][t] for t in synth.NTYPES])
        local = torch.arange(N) - offs[node_type]
        feats = synth.type_features(gd["counts"], {t: 128 for t in synth.NTYPES}, seed=1,
                                    device="cpu")
        x_dict = {k: f for k, f in enumerate(feats)}
        n_paper = gd["counts"]["paper"]
        y = torch.randint(0, classes, (N,), generator=torch.Generator().manual_seed(2))
        torch.manual_seed(3)
        model = REGNNCPU(128, hidden, classes, len(sizes), 10.0, 0.5, len(x_dict))
        model.train()
        opt = torch.optim.Adam(model.parameters(), lr=1e-3)
        smp = Sampler(ptr, idx, N)
        perm = np.random.default_rng(0).permutation(n_paper)
        times, edges = [], []
        for i in range(warm + steps):
            t0 = time.perf_counter()
            tg = perm[i * batch:(i + 1) * batch]
            n_id, adjs = smp.sample(tg, sizes, 123, 0, i)
            t_adjs = [(torch.from_numpy(s), torch.from_numpy(d), torch.from_numpy(p), sz)
                      for s, d, p, sz in adjs]
            opt.zero_grad()
            out = model(torch.from_numpy(n_id), x_dict, t_adjs, etype_csr, node_type, local)
            loss = F.nll_loss(out, y[torch.from_numpy(n_id[:len(tg)])])
            loss.backward()
            opt.step()
            dt = time.perf_counter() - t0
            if i >= warm:
                times.append(dt)
                edges.append(sum(s.size + sz[1] for s, _, _, sz in adjs))
        info = dict(N=N, E=int(idx.size), threads=torch.get_num_threads(), batch=batch,
                    sizes=list(sizes), hidden=hidden, classes=classes)
        return float(np.median(times)), float(np.median(edges)), info
    finally:
        torch.set_num_threads(prev)
