"""Graph-build host logic on CPU tensors (regnn_hip/graph.py): row offsets by binary search and
the relation histograms (short rows, long rows) against direct counts. No kernel is launched."""
import pytest
import torch

from regnn_hip.graph import RelGraph, RelPack


def _counts(keys, n):
    c = torch.bincount(keys, minlength=n)
    return torch.cat([c.new_zeros(1), torch.cumsum(c, 0)]).to(torch.int32)


@pytest.mark.parametrize("order", ["edge", "source"])
@pytest.mark.parametrize("n,E", [(1, 0), (7, 3), (300, 20000)])
def test_offsets_and_relation_histograms(order, n, E):
    g = torch.Generator().manual_seed(n + E)
    R = 7
    src = torch.randint(0, n, (E,), generator=g)
    dst = (torch.rand(E, generator=g) ** 4 * n).long().clamp(max=n - 1)   # skewed: hub rows
    e = torch.randint(1, R + 1, (E,), generator=g)
    rg = RelGraph(src, dst, n, "cpu", order=order, split=16, chunk=16)
    assert torch.equal(rg.csr_ptr, _counts(dst, n))
    assert torch.equal(rg.csc_ptr, _counts(src, n))
    rp = RelPack(rg, e, R)
    full = torch.zeros(n, R, dtype=torch.int64)
    full.index_put_((dst, e - 1), torch.ones(E, dtype=torch.int64), accumulate=True)
    plan = rg.csr_plan
    want = full.clone()
    if plan.n_long:
        want[plan.long_ids.long()] = 0
        assert torch.equal(rp.long_cnt(R).long(), full[plan.long_ids.long()])
    else:
        assert rp.long_cnt(R) is None
    assert torch.equal(rp.row_cnt(R).long(), want)


def test_out_of_range_node_ids_raise():
    with pytest.raises(ValueError, match="node ids"):
        RelGraph(torch.tensor([0, 1]), torch.tensor([0, 5]), 3, "cpu")
