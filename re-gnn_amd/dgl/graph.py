"""DGLGraph-compatible homogeneous graph whose message passing runs on the HIP kernels."""
import contextlib

import numpy as np
import torch

from .base import DGLError



# row order of the device layout (regnn_hip.graph): "source" sorts each row by the gathered id and
# schedules hub-row chunks by source range (shared rows hit in L2 / Infinity Cache); "edge" keeps
# DGL's edge-id summation order
RELGRAPH_ORDER = "source"

class _Frame(dict):
    pass


class _EdgeEnd(torch.Tensor):
    """One end of ``g.edges()`` on a device graph: the device id tensor (DGL semantics) whose Python
    iteration reads a host copy made once per graph, so run_regnn.py:94-99's per-edge
    ``u.cpu().item()`` loop costs no device round trip per edge. Tensor ops return plain tensors."""

    __torch_function__ = torch._C._disabled_torch_function_impl

    def __iter__(self):
        return iter(self._host)


class DGLGraph:
    """Directed multigraph in caller edge order (DGL semantics: edge e is src[e] -> dst[e]).

    Construction follows DGL 0.7: ``DGLGraph(scipy_matrix)`` makes one edge per stored entry
    (src = row, dst = col) in row-major order; ``DGLGraph((src, dst), num_nodes=N)`` takes explicit
    lists. The device layout (CSR/CSC, see regnn_hip.graph.RelGraph) is built lazily, once per
    device, and shared by ``local_var()`` views.
    """

    is_block = False

    def __init__(self, data=None, num_nodes=None, device=None):
        if data is None:
            src = torch.zeros(0, dtype=torch.int64)
            dst = torch.zeros(0, dtype=torch.int64)
        elif isinstance(data, tuple):
            src, dst = (torch.as_tensor(np.asarray(x) if not torch.is_tensor(x) else x)
                        .to(torch.int64).reshape(-1) for x in data)
        elif hasattr(data, "tocsr"):
            coo = data.tocsr().tocoo()
            src = torch.from_numpy(coo.row.astype(np.int64))
            dst = torch.from_numpy(coo.col.astype(np.int64))
            if num_nodes is None:
                num_nodes = max(data.shape)
        else:
            raise DGLError(f"unsupported graph data {type(data)}")
        if src.numel() != dst.numel():
            raise DGLError("src and dst must have the same length")
        if num_nodes is None:
            num_nodes = int(max(src.max().item(), dst.max().item()) + 1) if src.numel() else 0
        dev = torch.device(device) if device is not None else src.device
        self._src = src.to(dev)
        self._dst = dst.to(dev)
        self._n = int(num_nodes)
        self._rg_cache = {}
        self.ndata = _Frame()
        self.edata = _Frame()

    # ------------------------------------------------------------------ structure
    @property
    def device(self):
        return self._src.device

    @property
    def srcdata(self):
        return self.ndata

    @property
    def dstdata(self):
        return self.ndata

    def num_nodes(self, ntype=None):
        return self._n

    number_of_nodes = num_nodes

    def number_of_src_nodes(self):
        return self._n

    def number_of_dst_nodes(self):
        return self._n

    def num_edges(self, etype=None):
        return int(self._src.numel())

    number_of_edges = num_edges

    def edges(self, form="uv", order="eid"):
        if self._src.device.type == "cpu":
            return self._src, self._dst
        ends = self.__dict__.get("_edge_ends")
        if ends is None or ends[0]._host.numel() != self._src.numel():
            host = torch.stack([self._src, self._dst]).cpu()       # one copy, one sync
            ends = []
            for dev_ids, h in zip((self._src, self._dst), host):
                e = torch.Tensor._make_subclass(_EdgeEnd, dev_ids)
                e._host = h
                ends.append(e)
            self._edge_ends = ends = tuple(ends)
        return ends

    def in_degrees(self, v=None):
        deg = torch.bincount(self._dst, minlength=self._n)
        return deg if v is None else deg[v]

    def out_degrees(self, u=None):
        deg = torch.bincount(self._src, minlength=self._n)
        return deg if u is None else deg[u]

    def to(self, device, **kwargs):
        g = DGLGraph((self._src.to(device), self._dst.to(device)), num_nodes=self._n)
        if torch.device(device) == self.device:
            g._rg_cache = self._rg_cache
        g.ndata = _Frame({k: v.to(device) for k, v in self.ndata.items()})
        g.edata = _Frame({k: v.to(device) for k, v in self.edata.items()})
        return g

    def local_var(self):
        g = DGLGraph.__new__(DGLGraph)
        g._src, g._dst, g._n, g._rg_cache = self._src, self._dst, self._n, self._rg_cache
        g.ndata = _Frame(self.ndata)
        g.edata = _Frame(self.edata)
        return g

    @contextlib.contextmanager
    def local_scope(self):
        nd, ed = self.ndata, self.edata
        self.ndata, self.edata = _Frame(nd), _Frame(ed)
        try:
            yield
        finally:
            self.ndata, self.edata = nd, ed

    def relgraph(self, device=None):
        """the device CSR/CSC layout (regnn_hip.graph.RelGraph), built once per device."""
        from regnn_hip.graph import RelGraph
        dev = torch.device(device) if device is not None else self.device
        if dev.type != "cuda":
            raise DGLError("RE-GNN message passing runs on a ROCm device; move the graph and "
                           "features with .to('cuda') (there is no CPU path)")
        key = (dev.type, dev.index if dev.index is not None else torch.cuda.current_device())
        rg = self._rg_cache.get(key)
        if rg is None:
            rg = RelGraph(self._src, self._dst, self._n, dev, order=RELGRAPH_ORDER)
            self._rg_cache[key] = rg
        return rg

    # ------------------------------------------------------------------ message passing
    def update_all(self, message_func, reduce_func):
        from regnn_hip import ops
        m, r = message_func, reduce_func
        if r.msg != m.out:
            raise DGLError(f"reduce reads '{r.msg}' but the message writes '{m.out}'")
        x = self.ndata[m.lhs]
        rg = self.relgraph(x.device)
        if m.kind == "u_mul_e":
            w = self.edata[m.rhs]
            if w.numel() == rg.E:
                y = _flat_call(x, lambda x2: ops.edge_spmm(rg, x2, w.reshape(-1)))
            elif x.dim() == 3 and w.shape[0] == rg.E and w.numel() == rg.E * x.shape[1]:
                a = w.reshape(rg.E, x.shape[1])[rg.csr_eid]
                y = ops.head_spmm(rg, a, x)
            else:
                raise DGLError(f"u_mul_e: unsupported shapes {tuple(x.shape)} x {tuple(w.shape)}")
        elif m.kind == "copy_u":
            y = _flat_call(x, lambda x2: ops.re_spmm(rg, x2))
        else:
            raise DGLError(f"update_all: message {m.kind} not supported")
        if r.kind == "mean":
            inv = rg.inv_in_count().to(y.dtype)
            y = y * inv.view((-1,) + (1,) * (y.dim() - 1))
        elif r.kind != "sum":
            raise DGLError(f"reduce '{r.kind}' is not implemented on the HIP path")
        self.ndata[r.out] = y

    def apply_edges(self, func):
        if func.kind != "u_add_v":
            raise DGLError(f"apply_edges: {func.kind} not supported")
        self.edata[func.out] = self.ndata[func.lhs][self._src] + self.ndata[func.rhs][self._dst]


def _flat_call(x, fn):
    """run a row-SpMM on x reshaped to (N, F), F padded to a multiple of 8 (16-byte vectors)."""
    shape = x.shape
    x2 = x.reshape(shape[0], -1)
    F = x2.shape[1]
    pad = (-F) % 8
    if pad:
        x2 = torch.nn.functional.pad(x2, (0, pad))
    y = fn(x2)
    if pad:
        y = y[:, :F]
    return y.reshape((y.shape[0],) + tuple(shape[1:]))


def graph(data, num_nodes=None, device=None, **kwargs):
    return DGLGraph(data, num_nodes=num_nodes, device=device)


def remove_self_loop(g):
    keep = g._src != g._dst
    return DGLGraph((g._src[keep], g._dst[keep]), num_nodes=g._n)


def add_self_loop(g):
    """append one loop per node after the existing edges (loop ids E .. E+N-1, as DGL does)."""
    loop = torch.arange(g._n, device=g.device)
    return DGLGraph((torch.cat([g._src, loop]), torch.cat([g._dst, loop])), num_nodes=g._n)
