"""CPU ORACLE for the neighbour sampler — TEST INFRASTRUCTURE (tests / bench cpu leg only).

The reference samples with torch_sparse ``SparseTensor.sample_adj`` behind PyG ``NeighborSampler``
(mag/regnn_ns.py:206-214), whose RNG stream cannot be reproduced here (torch_sparse absent), so
parity for sampled indices is UNPINNED against the reference; this build defines its own
deterministic spec (include/regnn_hip.h), restated here in plain Python
integer arithmetic and required BIT-EXACT from the GPU sampler:

* in-neighbours of target t = CSR row t of the destination-major graph, in CSR (edge-id) order;
* deg <= k or k < 0: take all; else Floyd's algorithm over positions j = deg-k .. deg-1 with
  r_j = hash(seed, t, j) (splitmix64 finaliser below), pos = (r_j * (j+1)) >> 32,
  and the chosen positions emitted in ascending order;
* n_id of a hop = the hop's targets, then every newly seen source in first-seen order over the
  target-major candidate list (PyG sample_adj's n_id contract, mag/regnn_ns.py:399-401);
* block edge_index = [src_local, dst_local], e_id = CSR edge ids, size = (|n_id|, |targets|);
  adjs are returned outermost hop first (PyG NeighborSampler ``adjs[::-1]``);
* per-hop seed = mix(base_seed, epoch, batch, hop) (``hop_seed``).
"""
M64 = (1 << 64) - 1


def _mix(x):
    x &= M64
    x ^= x >> 30
    x = (x * 0xBF58476D1CE4E5B9) & M64
    x ^= x >> 27
    x = (x * 0x94D049BB133111EB) & M64
    x ^= x >> 31
    return x


def sample_hash(seed, t, j):
    x = (seed + 0x9E3779B97F4A7C15 * (t + 1) + 0xD1B54A32D192ED03 * (j + 1)) & M64
    return _mix(x) >> 32


def hop_seed(base, epoch, batch, hop):
    return _mix((base & M64) ^ _mix((epoch << 40) ^ (batch << 8) ^ hop))


def sample_row(ptr, idx, t, k, seed):
    b, e = int(ptr[t]), int(ptr[t + 1])
    d = e - b
    if k < 0 or d <= k:
        return [int(idx[b + q]) for q in range(d)], list(range(b, e))
    chosen = []
    for j in range(d - k, d):
        pos = (sample_hash(seed, t, j) * (j + 1)) >> 32
        chosen.append(j if pos in chosen else pos)
    chosen.sort()
    return [int(idx[b + p]) for p in chosen], [b + p for p in chosen]


def sample_hop(ptr, idx, n_id, k, seed):
    """one hop: returns (new n_id, src_local, dst_local, e_id)."""
    local = {int(g): i for i, g in enumerate(n_id)}
    new = list(n_id)
    src_l, dst_l, eids = [], [], []
    for i, t in enumerate(n_id):
        srcs, es = sample_row(ptr, idx, int(t), k, seed)
        for s, e in zip(srcs, es):
            if s not in local:
                local[s] = len(new)
                new.append(s)
            src_l.append(local[s])
            dst_l.append(i)
            eids.append(e)
    return new, src_l, dst_l, eids


def neighbor_sample(ptr, idx, batch, sizes, base_seed, epoch=0, batch_idx=0):
    """-> (batch_size, n_id, adjs) with adjs = [(src_local, dst_local, e_id, (n_src, n_dst))],
    outermost hop first."""
    n_id = [int(x) for x in batch]
    adjs = []
    for hop, k in enumerate(sizes):
        seed = hop_seed(base_seed, epoch, batch_idx, hop)
        n_dst = len(n_id)
        n_id, s, d, e = sample_hop(ptr, idx, n_id, k, seed)
        adjs.append((s, d, e, (len(n_id), n_dst)))
    return len(batch), n_id, adjs[::-1]
