"""Minimal homogeneous graph with DGL's frame semantics (test-only, see package docstring)."""
import contextlib

import numpy as np
import torch


class _Frame(dict):
    pass


class DGLGraph:
    def __init__(self, data=None, num_nodes=None):
        if data is None:
            src = torch.zeros(0, dtype=torch.long)
            dst = torch.zeros(0, dtype=torch.long)
        elif isinstance(data, tuple):
            src, dst = (torch.as_tensor(np.asarray(x), dtype=torch.long) for x in data)
        else:  # scipy sparse matrix: one edge per stored entry, src=row, dst=col, row-major
            coo = data.tocsr().tocoo()
            src = torch.as_tensor(coo.row.astype(np.int64))
            dst = torch.as_tensor(coo.col.astype(np.int64))
            num_nodes = data.shape[0]
        if num_nodes is None:
            num_nodes = int(max(src.max().item(), dst.max().item()) + 1) if src.numel() else 0
        self._src, self._dst, self._n = src, dst, int(num_nodes)
        self.ndata = _Frame()
        self.edata = _Frame()

    # --- structure -------------------------------------------------------------------------
    @property
    def srcdata(self):
        return self.ndata

    @property
    def dstdata(self):
        return self.ndata

    is_block = False

    def num_nodes(self):
        return self._n

    number_of_nodes = num_nodes

    def number_of_dst_nodes(self):
        return self._n

    def num_edges(self):
        return self._src.numel()

    def edges(self):
        return self._src, self._dst

    def in_degrees(self):
        return torch.bincount(self._dst, minlength=self._n)

    def to(self, device):
        return self

    def local_var(self):
        g = DGLGraph.__new__(DGLGraph)
        g._src, g._dst, g._n = self._src, self._dst, self._n
        g.ndata = _Frame(self.ndata)
        g.edata = _Frame(self.edata)
        return g

    @contextlib.contextmanager
    def local_scope(self):
        nd, ed = _Frame(self.ndata), _Frame(self.edata)
        try:
            yield
        finally:
            self.ndata, self.edata = nd, ed

    # --- message passing -------------------------------------------------------------------
    def _message(self, msg):
        if msg.kind == "u_mul_e":
            h = self.ndata[msg.a][self._src]
            w = self.edata[msg.b]
            while w.dim() < h.dim():
                w = w.unsqueeze(-1)
            return h * w
        if msg.kind == "copy_u":
            return self.ndata[msg.a][self._src]
        if msg.kind == "u_add_v":
            return self.ndata[msg.a][self._src] + self.ndata[msg.b][self._dst]
        raise NotImplementedError(msg.kind)

    def update_all(self, msg, red):
        m = self._message(msg)
        shape = (self._n,) + tuple(m.shape[1:])
        out = torch.zeros(shape, dtype=m.dtype).index_add(0, self._dst, m)
        if red.kind == "mean":
            cnt = torch.bincount(self._dst, minlength=self._n).clamp(min=1).to(m.dtype)
            out = out / cnt.view((-1,) + (1,) * (m.dim() - 1))
        elif red.kind == "max":
            idx = self._dst.view((-1,) + (1,) * (m.dim() - 1)).expand_as(m)
            out = torch.zeros(shape, dtype=m.dtype).scatter_reduce(0, idx, m, "amax",
                                                                   include_self=False)
        self.ndata[red.out] = out

    def apply_edges(self, msg):
        self.edata[msg.out] = self._message(msg)


def graph(data, num_nodes=None):
    return DGLGraph(data, num_nodes=num_nodes)


def remove_self_loop(g):
    keep = g._src != g._dst
    return DGLGraph((g._src[keep].numpy(), g._dst[keep].numpy()), num_nodes=g._n)


def add_self_loop(g):
    loop = torch.arange(g._n)
    return DGLGraph((torch.cat([g._src, loop]).numpy(), torch.cat([g._dst, loop]).numpy()),
                    num_nodes=g._n)
