"""Host-side helpers that run without a GPU: the chunked weight-gradient reduction used by the
HIP-path Linear / head backward must equal the plain g^T x."""
import torch

from regnn_hip import ops


def test_batched_wgrad_matches_mm():
    torch.manual_seed(0)
    for rows in (5, 4096, 3 * 4096 + 17):
        g = torch.randn(rows, 7, dtype=torch.float64)
        x = torch.randn(rows, 5, dtype=torch.float64)
        got = ops.batched_wgrad(g, x, chunk=1024)
        assert torch.allclose(got, g.t() @ x, rtol=1e-12, atol=1e-10)


def test_source_order_layout_and_chunk_schedule():
    """RelGraph(order="source") on the CPU: rows sorted by gathered id (ties by edge id), eid /
    csc2csr consistent, and the chunk schedule a permutation sorted by each chunk's first
    gathered row (the kernels' processing order; regnn_hip.h scheduled plan form)."""
    import numpy as np
    import torch
    from regnn_hip.graph import RelGraph
    rng = np.random.default_rng(0)
    N, E = 300, 6000
    src = rng.integers(0, N, E)
    dst = np.where(rng.random(E) < 0.5, 7, rng.integers(0, N, E))       # one hub row
    rg = RelGraph(src, dst, N, "cpu", split=16, chunk=8, order="source")
    s, d = torch.from_numpy(src), torch.from_numpy(dst)
    for ptr, idx, eid, key, other in ((rg.csr_ptr, rg.csr_idx, rg.csr_eid, d, s),
                                      (rg.csc_ptr, rg.csc_idx, rg.csc_eid, s, d)):
        assert torch.equal(key[eid], torch.repeat_interleave(torch.arange(N), ptr.diff()))
        assert torch.equal(other[eid].to(torch.int32), idx)
        for v in range(N):
            a, b = int(ptr[v]), int(ptr[v + 1])
            k = (idx[a:b].to(torch.int64) * E + eid[a:b])
            assert bool((k[1:] > k[:-1]).all())                 # by gathered id, ties by eid
    assert torch.equal(rg.csr_eid[rg.csc2csr.to(torch.int64)], rg.csc_eid)
    plan = rg.csr_plan
    n = plan.n_chunk
    sched = plan.chunk_sched
    assert sched.numel() == 2 * n and torch.equal(sched[:n], plan.chunk_long)
    order = sched[n:].to(torch.int64)
    assert torch.equal(torch.sort(order)[0], torch.arange(n))
    l = plan.chunk_long.to(torch.int64)[order]
    k = order - plan.chunk_off.to(torch.int64)[l]
    first = rg.csr_ptr.to(torch.int64)[plan.long_ids.to(torch.int64)[l]] + k * plan.chunk
    fs = rg.csr_idx[first]
    assert bool((fs[1:] >= fs[:-1]).all())
    assert RelGraph(src, dst, N, "cpu", split=16, chunk=8).csr_plan.chunk_sched is None


def test_csc_prefix_keeps_edges_into_leading_rows():
    """RelGraph.csc_prefix(n): per source, exactly the CSC edges with destination < n, in their
    CSC order, with the relation ids of those edges and a split plan of the shortened rows (the
    backward under the output head's zero gradient rows >= n, ops._ReSpmm)."""
    import numpy as np
    import torch
    from regnn_hip.graph import RelGraph
    rng = np.random.default_rng(1)
    N, E, n = 300, 6000, 120
    src = np.where(rng.random(E) < 0.4, 5, rng.integers(0, N, E))        # one long CSC row
    dst = rng.integers(0, N, E)
    rel = rng.integers(1, 8, E)
    for order in ("edge", "source"):
        rg = RelGraph(src, dst, N, "cpu", split=16, chunk=8, order=order)
        pack = rg.rel_pack(torch.from_numpy(rel), num_rel=7)
        pre = rg.csc_prefix(n)
        assert rg.csc_prefix(N) is None and rg.csc_prefix(n) is pre
        rc = pack.rel_csc_prefix(pre)
        assert pre.E == int((dst < n).sum()) == rc.numel()
        for u in range(N):
            a, b = int(rg.csc_ptr[u]), int(rg.csc_ptr[u + 1])
            m = rg.csc_idx[a:b] < n
            a2, b2 = int(pre.csc_ptr[u]), int(pre.csc_ptr[u + 1])
            assert torch.equal(pre.csc_idx[a2:b2], rg.csc_idx[a:b][m])
            assert torch.equal(rc[a2:b2], pack.rel_csc[a:b][m])
        deg = pre.csc_ptr.diff()
        assert torch.equal(pre.csc_plan.long_ids.to(torch.int64), torch.nonzero(deg > 16).flatten())
        assert (pre.csc_plan.chunk_sched is not None) == (order == "source")


def test_row_cnt_histogram():
    """RelPack.row_cnt: per CSR row the count of each relation among its in-edges, long rows
    (more than `split` edges) zero (regnn_degree_cnt's table)."""
    import numpy as np
    import torch
    from regnn_hip.graph import RelGraph
    rng = np.random.default_rng(2)
    N, E, R = 200, 5000, 6
    src = rng.integers(0, N, E)
    dst = np.where(rng.random(E) < 0.3, 9, rng.integers(0, N, E))        # row 9 is long
    rel = rng.integers(1, R + 1, E)
    rg = RelGraph(src, dst, N, "cpu", split=16, chunk=8)
    pack = rg.rel_pack(torch.from_numpy(rel), num_rel=R)
    cnt = pack.row_cnt(R)
    assert cnt.shape == (N, R) and cnt.dtype == torch.int16
    want = np.zeros((N, R), np.int64)
    np.add.at(want, (dst, rel - 1), 1)
    want[np.bincount(dst, minlength=N) > 16] = 0
    assert np.array_equal(cnt.numpy().astype(np.int64), want)


def test_fused_ns_gate_matches_kernel_limits():
    """ns.fused_unsupported refuses what regnn_nsm_step would reject (T * (K + 1) > 600 with
    K = 128 means at most 4 node types), so engine='auto' falls back to the module path instead
    of failing at the first step."""
    import torch
    from regnn_hip import mag, ns

    def gate(T, K):
        m = mag.REGNN(K, 64, 11, 2, 10.0, 0.0, {k: K for k in range(T)}, 7, use_norm="ln",
                      self_loop_type=2)
        return ns.fused_unsupported(m, {k: torch.zeros(3, K) for k in range(T)})
    assert gate(4, 128) is None
    assert gate(8, 64) is None
    assert gate(5, 128) is not None
    assert gate(2, 96) is not None
