"""Seeded synthetic multi-relation graphs of the BASELINE shapes (no datasets are available offline).

* ``mag_like(scale)`` — ogbn-mag-shaped heterogeneous graph: node types
  paper / author / institution / field at ``scale`` x ogbn-mag counts, the 4 raw relations at
  ``scale`` x counts plus their reverses (cites made undirected, mag/regnn_ns.py:93-105) = 7 edge
  types, + one self-loop type per node type = 11 relations. Destinations are Zipf(s=1.1)
  distributed inside their node type (power-law in-degree), sources uniform.
* ``dblp_like()`` — DBLP shape: A 4,057 / P 14,328 / T 7,723 / V 20,
  A-P 19,645, P-T 85,810, P-V 14,328 undirected, relation ids 1..6, self loops 6 + ntype + 1.

Edges come out in "DGL order" (relation blocks, then self loops appended, as
dgl.add_self_loop does); relation ids are 1-based as the reference's e_feat.
"""
import torch

MAG_NODES = {"paper": 736_389, "author": 1_134_649, "institution": 8_740, "field": 59_965}
MAG_EDGES = [  # (src type, dst type, count)  ogbn-mag raw relations
    ("author", "institution", 1_043_998),
    ("author", "paper", 7_145_660),
    ("paper", "paper", 5_416_271),
    ("paper", "field", 7_505_078),
]
NTYPES = ["paper", "author", "institution", "field"]


def _zipf(n, size, s, gen, device):
    u = torch.rand(size, generator=gen, device=device, dtype=torch.float64)
    a = 1.0 - s
    r = ((float(n) ** a - 1.0) * u + 1.0) ** (1.0 / a)
    return (r.floor().to(torch.int64) - 1).clamp_(0, n - 1)


def mag_like(scale=1.0, seed=0, device="cuda", zipf_s=1.1):
    """returns dict(src, dst, rel (1-based int64), ntype, type_offsets, N, R, counts)."""
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    counts = {t: max(1, int(round(c * scale))) for t, c in MAG_NODES.items()}
    off, o = {}, 0
    for t in NTYPES:
        off[t] = o
        o += counts[t]
    N = o
    perm = {t: torch.randperm(counts[t], generator=gen, device=device) for t in NTYPES}
    srcs, dsts, rels = [], [], []
    rid = 0
    blocks = []
    for st, dt, c in MAG_EDGES:
        m = max(1, int(round(c * scale)))
        s = torch.randint(0, counts[st], (m,), generator=gen, device=device)
        d = perm[dt][_zipf(counts[dt], m, zipf_s, gen, device)]
        blocks.append((s + off[st], d + off[dt]))
    # forward relations 1..4 (cites stored in both directions as one relation: to_undirected)
    for i, (s, d) in enumerate(blocks):
        rid = i + 1
        if i == 2:
            s, d = torch.cat([s, d]), torch.cat([d, s])
        srcs.append(s); dsts.append(d)
        rels.append(torch.full((s.numel(),), rid, dtype=torch.uint8, device=device))
    # reverse relations 5..7 for affiliated_with, writes, has_topic
    for j, i in enumerate((0, 1, 3)):
        s, d = blocks[i]
        srcs.append(d); dsts.append(s)
        rels.append(torch.full((s.numel(),), 5 + j, dtype=torch.uint8, device=device))
    ntype = torch.cat([torch.full((counts[t],), k, dtype=torch.int64, device=device)
                       for k, t in enumerate(NTYPES)])
    loops = torch.arange(N, device=device)
    srcs.append(loops); dsts.append(loops)
    rels.append((8 + ntype).to(torch.uint8))
    src = torch.cat(srcs)
    dst = torch.cat(dsts)
    rel = torch.cat(rels)
    return dict(src=src, dst=dst, rel=rel, ntype=ntype, N=N, R=11, counts=counts,
                type_offsets=off)


DBLP_NODES = {"A": 4_057, "P": 14_328, "T": 7_723, "V": 20}
DBLP_DIMS = {"A": 334, "P": 4_231, "T": 50, "V": 20}


def dblp_like(seed=0, device="cuda"):
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    order = ["A", "P", "T", "V"]
    off, o = {}, 0
    for t in order:
        off[t] = o
        o += DBLP_NODES[t]
    N = o
    nP = DBLP_NODES["P"]

    def rnd(t, m):
        return torch.randint(0, DBLP_NODES[t], (m,), generator=gen, device=device) + off[t]

    ap = (rnd("A", 19_645), rnd("P", 19_645))
    pt = (rnd("P", 85_810), rnd("T", 85_810))
    pv = (torch.arange(nP, device=device) + off["P"], rnd("V", nP))
    srcs, dsts, rels = [], [], []
    for k, (a, b) in enumerate((ap, pt, pv)):
        srcs += [a, b]; dsts += [b, a]
        rels += [torch.full((a.numel(),), 2 * k + 1, dtype=torch.uint8, device=device),
                 torch.full((a.numel(),), 2 * k + 2, dtype=torch.uint8, device=device)]
    ntype = torch.cat([torch.full((DBLP_NODES[t],), k, dtype=torch.int64, device=device)
                       for k, t in enumerate(order)])
    loops = torch.arange(N, device=device)
    srcs.append(loops); dsts.append(loops)
    rels.append((7 + ntype).to(torch.uint8))
    return dict(src=torch.cat(srcs), dst=torch.cat(dsts), rel=torch.cat(rels), ntype=ntype,
                N=N, R=10, counts=dict(DBLP_NODES), type_offsets=off)


def _bipartite_hetero(spec, counts, seed, device):
    """node types in `counts` order; spec = [(src type, dst type, n_edges, one_per_src)];
    relation ids: 2k+1 for spec k forward, 2k+2 reversed; self loops num_etype + ntype + 1."""
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    order = list(counts)
    off, o = {}, 0
    for t in order:
        off[t] = o
        o += counts[t]
    N = o
    srcs, dsts, rels = [], [], []
    for k, (st, dt, m, one) in enumerate(spec):
        a = (torch.arange(counts[st], device=device) if one else
             torch.randint(0, counts[st], (m,), generator=gen, device=device)) + off[st]
        b = torch.randint(0, counts[dt], (a.numel(),), generator=gen, device=device) + off[dt]
        srcs += [a, b]; dsts += [b, a]
        rels += [torch.full((a.numel(),), 2 * k + 1, dtype=torch.uint8, device=device),
                 torch.full((a.numel(),), 2 * k + 2, dtype=torch.uint8, device=device)]
    n_et = 2 * len(spec)
    ntype = torch.cat([torch.full((counts[t],), i, dtype=torch.int64, device=device)
                       for i, t in enumerate(order)])
    loops = torch.arange(N, device=device)
    srcs.append(loops); dsts.append(loops)
    rels.append((n_et + 1 + ntype).to(torch.uint8))
    return dict(src=torch.cat(srcs), dst=torch.cat(dsts), rel=torch.cat(rels), ntype=ntype, N=N,
                R=n_et + len(order), counts=dict(counts), type_offsets=off)


ACM_NODES = {"P": 4_019, "A": 7_167, "S": 60}
ACM_DIMS = {"P": 1_902, "A": 10, "S": 10}
IMDB_NODES = {"M": 4_278, "D": 2_081, "A": 5_257}
IMDB_DIMS = {"M": 3_066, "D": 10, "A": 10}


def acm_like(seed=0, device="cuda"):
    """ACM shape: P-A 13,407 and P-S (one subject per paper), both
    directions + self loops, R = 4 + 3 = 7."""
    return _bipartite_hetero([("P", "A", 13_407, False), ("P", "S", 4_019, True)], ACM_NODES,
                             seed, device)


def imdb_like(seed=0, device="cuda"):
    """IMDB shape: M-D (one director per movie) and M-A 12,828, both
    directions + self loops, R = 4 + 3 = 7."""
    return _bipartite_hetero([("M", "D", 4_278, True), ("M", "A", 12_828, False)], IMDB_NODES,
                             seed, device)


def type_features(counts, dims, seed=1, device="cuda", kind="mag"):
    """per-type dense input features (feats_type 3 for mag: paper N(0,1), others U(-0.5,0.5))."""
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    feats = []
    for i, (t, n) in enumerate(counts.items()):
        d = dims[t] if isinstance(dims, dict) else dims
        if kind == "mag":
            if i == 0:
                f = torch.randn(n, d, generator=gen, device=device)
            else:
                f = torch.rand(n, d, generator=gen, device=device) - 0.5
        elif kind == "target":   # feats_type 1: target type bag-of-words, zeros(10) for others
            f = ((torch.rand(n, d, generator=gen, device=device) < 0.01).float() if i == 0
                 else torch.zeros(n, d, device=device))
        else:  # dblp: binary bag-of-words A/P, gaussian T, identity V (utils/data.py:163-167)
            if t in ("A", "P"):
                f = (torch.rand(n, d, generator=gen, device=device) < 0.01).float()
            elif t == "T":
                f = torch.randn(n, d, generator=gen, device=device)
            else:
                f = torch.eye(n, d, device=device)
        feats.append(f)
    return feats
