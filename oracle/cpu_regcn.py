"""CPU BASELINE (test / bench infrastructure only: imported by tests/ and bench.py's cpu_baseline
leg, never by the product path).

A PyTorch CPU restatement of the REGraphConv stack's forward and backward
(layer/REGraphConv.py:52-106, weightless norm=True layers as REGCN's first and last,
model/REGCN.py:28,31) on fused ``torch.sparse`` CSR kernels (MKL SpMM for the aggregation and its
transpose, ``sampled_addmm`` for the per-edge SDDMM dot, ``segment_reduce`` for the weighted
degree) — the CPU plan of BASELINE.md §3. The reference's own DGL/PyG CPU path cannot run here
(DGL / PyG absent, reference code does not travel), so this is the "port" baseline; it is pinned
to the golden vectors of the shim-run reference in tests/test_cpu_baseline.py.
"""
import numpy as np
import torch


class CsrGraph:
    """CSR by destination + its transpose, built once (untimed); per-edge values move between
    the two orders through ``t_perm``."""

    def __init__(self, src, dst, N):
        src = torch.as_tensor(src, dtype=torch.int64)
        dst = torch.as_tensor(dst, dtype=torch.int64)
        self.N = int(N)
        order = torch.sort(dst * self.N + src, stable=True)[1]
        self.eid = order                                   # CSR position -> caller edge id
        self.col = src[order].contiguous()
        self.row = dst[order].contiguous()
        self.crow = torch.zeros(self.N + 1, dtype=torch.int64)
        self.crow[1:] = torch.cumsum(torch.bincount(self.row, minlength=self.N), 0)
        t = torch.sort(self.col * self.N + self.row, stable=True)[1]
        self.t_perm = t                                    # transpose position -> CSR position
        self.t_col = self.row[t].contiguous()
        self.t_crow = torch.zeros(self.N + 1, dtype=torch.int64)
        self.t_crow[1:] = torch.cumsum(torch.bincount(self.col, minlength=self.N), 0)
        self.E = int(src.numel())

    def mats(self, ew_csr):
        A = torch.sparse_csr_tensor(self.crow, self.col, ew_csr, (self.N, self.N))
        At = torch.sparse_csr_tensor(self.t_crow, self.t_col, ew_csr[self.t_perm].contiguous(),
                                     (self.N, self.N))
        return A, At


def _lrelu(v):
    return torch.where(v >= 0, v, 0.01 * v)


class REGraphConvCPU:
    """one weightless REGraphConv(norm=True) layer: forward + explicit backward."""

    def __init__(self, alpha):
        self.alpha = float(alpha)

    def forward(self, g, x, rel_csr, w):
        tab = _lrelu(self.alpha * w.reshape(-1))                       # :58-60
        ew = tab[rel_csr]                                               # :61
        deg = torch.segment_reduce(ew, "sum", offsets=g.crow)           # :66-69
        norm = deg.clamp(min=1).pow(-0.5)                               # :70-72
        h = x * norm[:, None]                                           # :73-76
        A, At = g.mats(ew)
        rst = A @ h                                                     # :84-86
        out = rst * norm[:, None]                                       # :97-98
        self.cache = (x, w, tab, deg, norm, h, rst, At, rel_csr)
        return out

    def backward(self, g, gout):
        x, w, tab, deg, norm, h, rst, At, rel_csr = self.cache
        g_rst = gout * norm[:, None]
        g_h = At @ g_rst
        gx = g_h * norm[:, None]
        g_norm = (gout * rst).sum(1) + (g_h * x).sum(1)
        dc = deg.clamp(min=1)
        g_deg = g_norm * (-0.5) * dc.pow(-1.5) * (deg >= 1).to(deg.dtype)
        pattern = torch.sparse_csr_tensor(g.crow, g.col, torch.ones(g.E, dtype=x.dtype),
                                          (g.N, g.N))
        dots = torch.sparse.sampled_addmm(pattern, g_rst, h.t(), beta=0.0).values()
        g_ew = dots + g_deg[g.row]
        g_tab = torch.zeros(tab.numel(), dtype=x.dtype).index_add_(0, rel_csr, g_ew)
        v = self.alpha * w.reshape(-1)
        g_w = g_tab * self.alpha * torch.where(v >= 0, 1.0, 0.01).to(x.dtype)
        return gx, g_w.view_as(w)


def regcn_stack_step(g, layers, x, rel_csr, ws):
    """forward + backward of the stack with gout = the output (the timed unit of the baseline)."""
    h = x
    for lay, w in zip(layers, ws):
        h = lay.forward(g, h, rel_csr, w)
    gx = h
    gws = []
    for lay in reversed(layers):
        gx, gw = lay.backward(g, gx)
        gws.append(gw)
    return h, gx, gws[::-1]


def rel_csr_of(g, rel):
    """0-based relation ids (reference e_feat - 1) in CSR order."""
    return (torch.as_tensor(np.asarray(rel), dtype=torch.int64)[g.eid] - 1).contiguous()
