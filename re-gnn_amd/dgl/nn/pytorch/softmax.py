"""dgl.nn.pytorch.softmax.edge_softmax for arbitrary per-edge logits (REGATv2Conv path).

REGATConv does not come through here: its attention is one fused HIP kernel
(regnn_hip.ops.gat_attention). This generic form serves other callers with device tensor ops.
"""
import torch

from ...base import DGLError


def edge_softmax(graph, logits, eids="__ALL__", norm_by="dst"):
    if norm_by != "dst":
        raise DGLError("edge_softmax: only norm_by='dst' is supported")
    if not logits.is_cuda:
        raise DGLError("edge_softmax runs on a ROCm device (no CPU path)")
    dst = graph._dst
    n = graph.num_nodes()
    idx = dst.view((-1,) + (1,) * (logits.dim() - 1)).expand_as(logits)
    shape = (n,) + tuple(logits.shape[1:])
    mx = torch.full(shape, float("-inf"), dtype=logits.dtype, device=logits.device)
    mx = mx.scatter_reduce(0, idx, logits.detach(), "amax", include_self=True)
    ex = torch.exp(logits - mx[dst])
    s = torch.zeros(shape, dtype=logits.dtype, device=logits.device).index_add(0, dst, ex)
    return ex / s[dst]
