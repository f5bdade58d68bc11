"""On-disk formats + vectorised graph construction (regnn_hip/data.py):
synthetic graphs of the BASELINE shapes written in the preprocessed layout utils/data.py reads,
loaded back, and the vectorised run_regnn.py:84-99 build compared with the reference's own
per-edge construction restated here (DGLGraph(adjM) -> remove_self_loop -> add_self_loop ->
e_feat[e] = adjMM_wsl_2[(u, v)] in a Python loop)."""
import numpy as np
import pytest
import scipy.sparse as sp
import torch

import dgl
from regnn_hip import data, synth


def _reference_build(adjM, adjMM_wsl_2):
    g = dgl.DGLGraph(adjM)
    g = dgl.remove_self_loop(g)
    g = dgl.add_self_loop(g)
    e_feat = []
    for u, v in zip(*g.edges()):                       # run_regnn.py:94-99
        u = u.cpu().item()
        v = v.cpu().item()
        e_feat.append(adjMM_wsl_2[(u, v)])
    return g, torch.tensor(e_feat, dtype=torch.long)


@pytest.mark.parametrize("dataset,make,n_types", [("ACM", synth.acm_like, 3),
                                                  ("IMDB", synth.imdb_like, 3)])
def test_roundtrip_and_vectorised_build(tmp_path, dataset, make, n_types):
    gd = make(seed=0, device="cpu")
    N = gd["N"]
    num_etype = int(gd["R"]) - n_types
    adjM, adjMM, adjMM_wsl, wsl2 = data.matrices_from_edges(
        gd["src"].numpy(), gd["dst"].numpy(), gd["rel"].numpy(), N, num_etype)
    rng = np.random.default_rng(0)
    counts = list(gd["counts"].values())
    feats = [rng.standard_normal((c, 8)).astype(np.float32) for c in counts]
    labels = rng.integers(0, 3, counts[0])
    tvt = {"train_idx": np.arange(0, counts[0], 2), "val_idx": np.arange(1, counts[0], 4),
           "test_idx": np.arange(3, counts[0], 4)}
    prefix = str(tmp_path / f"{dataset}_processed")
    data.save_preprocessed(prefix, dataset, feats, adjM, adjMM, adjMM_wsl, wsl2,
                           gd["ntype"].numpy(), labels, tvt)
    _, f2, adjM2, adjMM2, _, wsl2b, tm, lab, tvt2 = data.load_data(dataset, prefix)
    assert all(np.array_equal(a, b) for a, b in zip(f2, feats))
    assert (adjM2 != adjM).nnz == 0 and (wsl2b != wsl2).nnz == 0
    assert np.array_equal(lab, labels) and set(tvt2) == set(tvt)
    g, e_feat = data.build_graph(adjM2, wsl2b)
    g_ref, e_ref = _reference_build(adjM2, wsl2b)
    s, d = g.edges()
    s_ref, d_ref = g_ref.edges()
    assert torch.equal(s.cpu(), s_ref.cpu()) and torch.equal(d.cpu(), d_ref.cpu())
    assert torch.equal(e_feat.cpu(), e_ref)
    assert int(e_feat.min()) >= 1 and int(e_feat.max()) <= int(gd["R"])


def test_csr_lookup_absent_and_duplicates():
    m = sp.csr_matrix((np.array([1.0, 2.0, 5.0]), (np.array([0, 0, 2]), np.array([1, 1, 0]))),
                      shape=(3, 3))
    got = data.csr_lookup(m, [0, 2, 1, 0], [1, 0, 1, 0])
    assert got.tolist() == [3.0, 5.0, 0.0, 0.0]          # duplicates summed, absent -> 0


def test_edge_end_iterates_host_copy_and_ops_return_plain_tensors():
    """dgl.graph._EdgeEnd (what g.edges() returns on a device graph): iteration reads the host
    copy (run_regnn.py:94-99's loop costs no device round trip per edge); every tensor op gives a
    plain tensor. Checked here on host tensors; tests/test_gpu_configs.py checks the device case."""
    from dgl.graph import _EdgeEnd
    ids = torch.tensor([3, 1, 4, 1, 5])
    e = torch.Tensor._make_subclass(_EdgeEnd, ids)
    e._host = ids.clone() + 10                      # distinguishable from the tensor's data
    assert [int(u.item()) for u in e] == [13, 11, 14, 11, 15]
    assert type(e + 0) is torch.Tensor and type(e[1:]) is torch.Tensor
    assert torch.equal(e + 0, ids) and e.data_ptr() == ids.data_ptr()
