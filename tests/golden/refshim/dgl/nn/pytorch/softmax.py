"""Per-destination, max-subtracted edge softmax (DGL 0.7 ``edge_softmax`` semantics)."""
import torch


def edge_softmax(graph, logits, eids="__ALL__", norm_by="dst"):
    dst = graph._dst
    n = graph.num_nodes()
    idx = dst.view((-1,) + (1,) * (logits.dim() - 1)).expand_as(logits)
    shape = (n,) + tuple(logits.shape[1:])
    mx = torch.zeros(shape, dtype=logits.dtype).scatter_reduce(0, idx, logits, "amax",
                                                                include_self=False)
    ex = torch.exp(logits - mx[dst])
    s = torch.zeros(shape, dtype=logits.dtype).index_add(0, dst, ex)
    return ex / s[dst]
