"""TEST-ONLY torch_scatter subset (scatter sum/mean; the golden generator only)."""
import torch


def scatter(src, index, dim=0, dim_size=None, reduce="sum"):
    assert dim == 0
    n = int(index.max()) + 1 if dim_size is None else dim_size
    out = torch.zeros((n,) + tuple(src.shape[1:]), dtype=src.dtype).index_add(0, index, src)
    if reduce == "mean":
        cnt = torch.bincount(index, minlength=n).clamp(min=1).to(src.dtype)
        out = out / cnt.view((-1,) + (1,) * (src.dim() - 1))
    elif reduce != "sum":
        raise NotImplementedError(reduce)
    return out


def segment_csr(*a, **k):
    raise NotImplementedError


def gather_csr(*a, **k):
    raise NotImplementedError
