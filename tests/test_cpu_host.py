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
