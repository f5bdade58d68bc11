"""On-disk formats and graph construction of the full-batch harness.

* ``load_data(dataset, prefix)`` reads the MAGNN-style preprocessed directories that
  utils/data.py:19-185 reads (``adjM.npz``, ``adjMM*.npz``, ``adjMM_wsl*.npz``, ``features_*``,
  ``node_types.npy``, ``labels.npy``, ``train_val_test_idx.npz``) and returns the same 9-tuple.
  Every file goes through ``scipy.sparse.load_npz`` / ``numpy.load`` with pickles refused.
* ``build_graph(adjM, adjMM_wsl_2)`` is run_regnn.py:84-99 without the per-edge Python loop:
  ``DGLGraph(adjM)`` -> ``remove_self_loop`` -> ``add_self_loop`` and the relation id of every
  edge looked up in ``adjMM_wsl_2`` with one sorted-key search (O(E log E) in numpy instead of
  E interpreter iterations of scipy element access).
* ``save_preprocessed(...)`` writes the same layout (used to round-trip synthetic graphs of the
  BASELINE shapes through the loader, since the real datasets are not available offline).
"""
import os

import numpy as np
import scipy.sparse as sp
import torch

_ADJMM_NAME = {"DBLP": "adjMM.npz", "ACM": "adjMM_rgcn.npz", "IMDB": "adjMM.npz"}
_METAPATHS = {"DBLP": ["adj_010", "adj_01210", "adj_01310"], "ACM": ["adj_010", "adj_020"],
              "IMDB": ["adj_010", "adj_020"]}
_N_FEATS = {"DBLP": 4, "ACM": 3, "IMDB": 3}


def default_prefix(dataset):
    return f"data/preprocessed/{dataset}_processed"


def _npz(path):
    return sp.load_npz(path) if os.path.exists(path) else None


def load_data(dataset, prefix=None):
    """utils/data.py:load_data -> (metapath adjs, features_list, adjM, adjMM, adjMM_wsl,
    adjMM_wsl_2, type_mask, labels, train_val_test_idx). Features are dense float32 arrays
    (DBLP's venue features are eye(20), utils/data.py:167); missing metapath files are None."""
    if dataset not in _N_FEATS:
        raise ValueError(f"Invalid dataset {dataset!r} (DBLP, ACM, IMDB)")
    prefix = prefix or default_prefix(dataset)
    j = lambda name: os.path.join(prefix, name)  # noqa: E731
    metas = [_npz(j(m + ".npz")) for m in _METAPATHS[dataset]]
    feats = []
    for i in range(_N_FEATS[dataset]):
        if dataset == "DBLP" and i == 3:
            feats.append(np.eye(20, dtype=np.float32))
        elif dataset == "DBLP" and i == 2:
            feats.append(np.load(j("features_2.npy"), allow_pickle=False).astype(np.float32))
        else:
            feats.append(np.asarray(sp.load_npz(j(f"features_{i}.npz")).toarray(), np.float32))
    adjM = sp.load_npz(j("adjM.npz"))
    adjMM = sp.load_npz(j(_ADJMM_NAME[dataset]))
    adjMM_wsl = sp.load_npz(j("adjMM_wsl.npz"))
    adjMM_wsl_2 = sp.load_npz(j("adjMM_wsl_2.npz"))
    type_mask = np.load(j("node_types.npy"), allow_pickle=False)
    labels = np.load(j("labels.npy"), allow_pickle=False)
    with np.load(j("train_val_test_idx.npz"), allow_pickle=False) as z:
        tvt = {k: z[k] for k in z.files}
    return metas, feats, adjM, adjMM, adjMM_wsl, adjMM_wsl_2, type_mask, labels, tvt


def save_preprocessed(prefix, dataset, features_list, adjM, adjMM, adjMM_wsl, adjMM_wsl_2,
                      type_mask, labels, train_val_test_idx):
    """write the layout load_data reads (metapath adjacencies are not written)."""
    os.makedirs(prefix, exist_ok=True)
    j = lambda name: os.path.join(prefix, name)  # noqa: E731
    for i, f in enumerate(features_list):
        if dataset == "DBLP" and i == 3:
            continue
        if dataset == "DBLP" and i == 2:
            np.save(j("features_2.npy"), np.asarray(f, np.float32))
        else:
            sp.save_npz(j(f"features_{i}.npz"), sp.csr_matrix(np.asarray(f, np.float32)))
    sp.save_npz(j("adjM.npz"), sp.csr_matrix(adjM))
    sp.save_npz(j(_ADJMM_NAME[dataset]), sp.csr_matrix(adjMM))
    sp.save_npz(j("adjMM_wsl.npz"), sp.csr_matrix(adjMM_wsl))
    sp.save_npz(j("adjMM_wsl_2.npz"), sp.csr_matrix(adjMM_wsl_2))
    np.save(j("node_types.npy"), np.asarray(type_mask))
    np.save(j("labels.npy"), np.asarray(labels))
    np.savez(j("train_val_test_idx.npz"), **train_val_test_idx)


def matrices_from_edges(src, dst, rel, N, num_etype):
    """adjM / adjMM / adjMM_wsl_2 of a typed edge list whose self loops carry ids > num_etype
    (the synthetic generators' layout): adjM has the non-loop edges, adjMM their relation ids,
    adjMM_wsl_2 adds the per-node-type self-loop ids on the diagonal."""
    src, dst, rel = (np.asarray(a, np.int64) for a in (src, dst, rel))
    loop = src == dst
    e = ~loop
    adjM = sp.csr_matrix((np.ones(int(e.sum()), np.float32), (src[e], dst[e])), shape=(N, N))
    # relation ids are integer entries (run_regnn.py:98 builds a LongTensor from them); a
    # duplicated (u, v) pair keeps one id, as a preprocessed relation matrix holds
    uv = src * np.int64(N) + dst
    _, first = np.unique(uv, return_index=True)
    s1, d1, r1 = src[first], dst[first], rel[first]
    e1 = s1 != d1
    adjMM = sp.csr_matrix((r1[e1], (s1[e1], d1[e1])), shape=(N, N), dtype=np.int64)
    wsl2 = sp.csr_matrix((r1, (s1, d1)), shape=(N, N), dtype=np.int64)
    return adjM, adjMM, adjMM, wsl2


def csr_lookup(mat, rows, cols):
    """mat[rows[i], cols[i]] for every i (0 where absent), vectorised (scipy element access
    semantics: duplicate entries summed)."""
    m = sp.csr_matrix(mat)
    m.sum_duplicates()
    m.sort_indices()
    ncol = np.int64(m.shape[1])
    row_of = np.repeat(np.arange(m.shape[0], dtype=np.int64), np.diff(m.indptr))
    keys = row_of * ncol + m.indices.astype(np.int64)
    q = np.asarray(rows, np.int64) * ncol + np.asarray(cols, np.int64)
    pos = np.searchsorted(keys, q)
    pos_c = np.minimum(pos, max(keys.size - 1, 0))
    hit = (pos < keys.size) & (keys[pos_c] == q) if keys.size else np.zeros(q.shape, bool)
    out = np.zeros(q.shape, dtype=m.data.dtype)
    out[hit] = m.data[pos_c[hit]]
    return out


def build_graph(adjM, adjMM_wsl_2, device=None):
    """run_regnn.py:84-99 vectorised -> (dgl.DGLGraph on `device`, e_feat int64 [E])."""
    import dgl
    coo = sp.csr_matrix(adjM).tocoo()           # DGLGraph(adjM): one edge per stored entry
    src = coo.row.astype(np.int64)
    dst = coo.col.astype(np.int64)
    keep = src != dst                           # dgl.remove_self_loop
    N = int(max(adjM.shape))
    loops = np.arange(N, dtype=np.int64)        # dgl.add_self_loop appends loops 0..N-1
    src = np.concatenate([src[keep], loops])
    dst = np.concatenate([dst[keep], loops])
    e_feat = csr_lookup(adjMM_wsl_2, src, dst).astype(np.int64)     # adjMM_wsl_2[(u, v)]
    g = dgl.DGLGraph((src, dst), num_nodes=N)
    if device is not None:
        g = g.to(device)
    return g, torch.from_numpy(e_feat).to(device if device is not None else "cpu")


def loss_rows_first(num_nodes, train_idx, first_type_count):
    """node renumbering that puts the loss rows (train_idx, all of the first node type, as the
    target type of run_regnn.py / mag/regnn_ns.py is) at [0, n_train), the rest of the first
    type after them, every other node where it was: ops.head_ce's fast path (the loss rows a
    prefix) for any train split. Returns (perm, inv) int64: new row r holds old node perm[r],
    old node u becomes inv[u]. Apply once to the edge list (inv[src], inv[dst]), the first type's
    feature rows (x0[perm[:first_type_count]]) and the labels (labels[train_idx])."""
    t = torch.as_tensor(train_idx).reshape(-1).to(torch.int64)
    dev = t.device
    if t.numel() and (int(t.min()) < 0 or int(t.max()) >= first_type_count):
        raise ValueError("loss rows must lie in the first node type's range")
    is_train = torch.zeros(first_type_count, dtype=torch.bool, device=dev)
    is_train[t] = True
    if int(is_train.sum()) != t.numel():
        raise ValueError("duplicate loss rows")
    rest = torch.nonzero(~is_train).flatten()
    perm = torch.cat([torch.sort(t)[0], rest,
                      torch.arange(first_type_count, num_nodes, dtype=torch.int64, device=dev)])
    inv = torch.empty_like(perm)
    inv[perm] = torch.arange(num_nodes, dtype=torch.int64, device=dev)
    return perm, inv
