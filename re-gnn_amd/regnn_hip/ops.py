"""Autograd operators over the C-ABI (include/regnn_hip.h). Every forward and backward runs in the
HIP library on torch's current stream; torch only allocates buffers and does the R-sized table
math (LeakyReLU of the relation embedding) and dense projections.

* degree_norm(rg, pack, tab, power)           layer/REGraphConv.py:66-75
* re_spmm(rg, x, tab, pack, pre, post)         layer/REGraphConv.py:76,84-98 / REMixHopConv.py:78-82
                                               / mag/regnn_layers.py:129,142-148
* edge_spmm(rg, x, ew)                         generic fn.u_mul_e(h, ew) + fn.sum, ew per edge
* gat_attention(rg, el, er, ee_tab, pack, s)   layer/REGATConv.py:80-88
* head_spmm(rg, a, ft)                         layer/REGATConv.py:90-91
"""
import ctypes
import os

import torch

from . import _lib as L
from .profile import timed

_SLAB = None


def _slab(width, device):
    return torch.zeros(L.slab_rows(), width, dtype=torch.float32, device=device)


def _reduce(slab, width, out=None, accumulate=False):
    if out is None:
        out = torch.empty(width, dtype=torch.float32, device=slab.device)
    L.call("regnn_rel_reduce", L.ptr(slab), slab.shape[0], width, L.ptr(out), int(accumulate),
           L.stream())
    return out


class _SegPlanC(ctypes.Structure):
    """regnn_seg_plan (include/regnn_hip.h): a SegPlan for the GAT / per-head kernels."""
    _fields_ = [("split", ctypes.c_int32), ("chunk", ctypes.c_int32),
                ("long_ids", ctypes.c_void_p), ("n_long", ctypes.c_int32),
                ("chunk_long", ctypes.c_void_p), ("chunk_off", ctypes.c_void_p),
                ("n_chunk", ctypes.c_int32), ("level_sb", ctypes.c_void_p),
                ("n_levels", ctypes.c_int32), ("level_desc", ctypes.c_void_p),
                ("partial_rows", ctypes.c_int64), ("partial", ctypes.c_void_p),
                ("partial_floats", ctypes.c_int64)]


class _GatPlan:
    """a SegPlan as the C struct, with a partial buffer `width` floats wide (0: none). .ptr is
    the struct's address (None: no long segments); the object keeps the buffers alive."""

    def __init__(self, plan, width, device):
        self.ptr, self.part = None, None
        if plan is None or plan.n_chunk == 0:
            return
        if width:
            self.part = torch.empty(plan.partial_rows * width, dtype=torch.float32,
                                    device=device)
        self.c = _SegPlanC(plan.split, plan.chunk, L.ptr(plan.long_ids), plan.n_long,
                           L.ptr(plan.chunk_long), L.ptr(plan.chunk_off), plan.n_chunk,
                           L.ptr(plan.level_sb), plan.n_levels,
                           ctypes.cast(plan.level_desc, ctypes.c_void_p), plan.partial_rows,
                           L.ptr(self.part), 0 if self.part is None else self.part.numel())
        self.plan = plan
        self.ptr = ctypes.addressof(self.c)


def _plan_args(plan, F, device):
    if plan.n_chunk == 0:
        return (0, 0, None, 0, None, None, 0, None, None, 0, None), None
    part = plan.partial(F, device)
    if plan.chunk_sched is not None:
        # scheduled form (regnn_hip.h): chunk_long + the processing order, split negated
        return (-plan.split, plan.chunk, L.ptr(plan.long_ids), plan.n_long,
                L.ptr(plan.chunk_sched), L.ptr(plan.chunk_off), plan.n_chunk, L.ptr(part),
                L.ptr(plan.level_sb), plan.n_levels,
                ctypes.cast(plan.level_desc, ctypes.c_void_p)), part
    return (plan.split, plan.chunk, L.ptr(plan.long_ids), plan.n_long, L.ptr(plan.chunk_long),
            L.ptr(plan.chunk_off), plan.n_chunk, L.ptr(part), L.ptr(plan.level_sb),
            plan.n_levels, ctypes.cast(plan.level_desc, ctypes.c_void_p)), part


def spmm_bytes(E, n_dst, n_src, F, s, kind):
    """algorithmic HBM bytes of one SpMM launch: int32 ids, uint8 relation ids,
    fp32 norms. fwd: gather row + id + rel + norm[src] per edge; ptr, norm, out row per node.
    bwd: gather g row + id + rel + norm per edge; x, g, gx rows + ptr, norm, node grad per node
    (the kernel also reads y when forming the norm gradient: not credited)."""
    if kind == "spmm_fwd":
        return E * (F * s + 9) + n_dst * (F * s + 8)
    return E * (F * s + 9) + n_src * (3 * F * s + 12)


def _flat_table(tab):
    return None if tab is None else tab.detach().reshape(-1).to(torch.float32).contiguous()


# ---------------------------------------------------------------------------------------------
class _DegreeNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, tab, rg, pack, power):
        ctx.set_materialize_grads(False)
        dev = rg.device
        deg = torch.empty(rg.n_dst, dtype=torch.float32, device=dev)
        norm = torch.empty_like(deg)
        t = _flat_table(tab)
        n_rel = t.numel() if t is not None else 0
        plan = rg.csr_plan
        cnt = pack.long_cnt(n_rel) if (t is not None and plan.n_long) else None
        ctx.hist = _use_row_cnt(pack, t, n_rel)
        if ctx.hist:
            with timed("degree", rg.n_dst * (2 * n_rel + 8)):
                L.call("regnn_degree_cnt", L.ptr(pack.row_cnt(n_rel)), L.ptr(t), n_rel,
                       rg.n_dst, float(power), L.ptr(rg.csr_ptr), L.ptr(plan.long_ids),
                       plan.n_long if plan.split > 0 else 0, L.ptr(cnt), L.ptr(deg),
                       L.ptr(norm), L.stream())
        else:
            with timed("degree", rg.E + rg.n_dst * 16):
                L.call("regnn_degree", L.ptr(rg.csr_ptr), L.ptr(pack.rel_csr if pack else None),
                       L.ptr(t), rg.n_dst, float(power), plan.split,
                       L.ptr(plan.long_ids), plan.n_long, L.ptr(cnt), n_rel, L.ptr(deg),
                       L.ptr(norm), L.stream())
        ctx.rg, ctx.pack, ctx.power, ctx.n_rel, ctx.shape = rg, pack, power, n_rel, tab.shape
        ctx.save_for_backward(deg)
        ctx.mark_non_differentiable(deg)
        return norm, deg

    @staticmethod
    def backward(ctx, g_norm, _g_deg):
        if not ctx.needs_input_grad[0] or g_norm is None:
            return None, None, None, None
        (deg,) = ctx.saved_tensors
        rg, pack, n_rel = ctx.rg, ctx.pack, ctx.n_rel
        plan = rg.csr_plan
        slab = _slab(n_rel, rg.device)
        cnt = pack.long_cnt(n_rel) if plan.n_long else None
        if ctx.hist:
            with timed("degree_bwd", rg.n_dst * (2 * n_rel + 8)):
                L.call("regnn_degree_cnt_bwd", L.ptr(pack.row_cnt(n_rel)), L.ptr(deg),
                       L.ptr(g_norm.contiguous().float()), rg.n_dst, float(ctx.power), n_rel,
                       L.ptr(plan.long_ids), plan.n_long if plan.split > 0 else 0, L.ptr(cnt),
                       L.ptr(slab), L.stream())
        else:
            with timed("degree_bwd", rg.E + rg.n_dst * 16):
                L.call("regnn_degree_bwd", L.ptr(rg.csr_ptr), L.ptr(pack.rel_csr), L.ptr(deg),
                       L.ptr(g_norm.contiguous().float()), rg.n_dst, float(ctx.power), n_rel,
                       plan.split, L.ptr(plan.long_ids), plan.n_long, L.ptr(cnt), L.ptr(slab),
                       L.stream())
        g = _reduce(slab, n_rel)
        return g.view(ctx.shape), None, None, None


# "hist": weighted degrees from the per-row relation histogram (RelPack.row_cnt,
# regnn_degree_cnt), built once per graph; "off": walk the relation ids every call
DEGREE = {"mode": os.environ.get("REGNN_DEGREE", "hist")}


def _use_row_cnt(pack, t, n_rel):
    return (DEGREE["mode"] == "hist" and pack is not None and t is not None and
            0 < n_rel <= 16 and pack.max_rel <= n_rel and pack.rg.device.type == "cuda")


def degree_norm(rg, pack, tab, power=-0.5):
    """norm[v] = max(sum_{e->v} tab[rel_e], 1)^power  (differentiable in tab)."""
    norm, _ = _DegreeNorm.apply(tab, rg, pack, power)
    return norm


def in_count_norm(rg, power=-0.5):
    """unweighted variant (copy_u degree)."""
    deg = rg.in_degree().to(torch.float32)
    return deg.clamp(min=1).pow(power)


# ---------------------------------------------------------------------------------------------
_DROP_CTR = {}


def dropout_fusable(x):
    """the fused-dropout SpMM kernels take rows of 8 or 16 16-byte vectors (F = 64 fp32 / 64 or
    128 bf16)."""
    return x.is_cuda and x.dim() == 2 and x.shape[1] * x.element_size() in (128, 256) and \
        x.dtype in (torch.float32, torch.bfloat16)


def drop_request(p, device, seed=None):
    """one fused-dropout call: (seed tensor on the device, 16-bit keep threshold, scale).

    The seed is a fresh device scalar per call, derived from a per-device counter whose base is
    drawn from torch's CPU generator (so torch.manual_seed makes runs repeatable); the counter
    increment is a device op, so a captured HIP graph draws a new mask on every replay."""
    keep = 1.0 - float(p)
    if seed is None:
        ctr = _DROP_CTR.get(device)
        if ctr is None:
            base = int(torch.randint(1, 2 ** 62, (1,)).item())
            ctr = _DROP_CTR[device] = torch.tensor([base], dtype=torch.int64, device=device)
        ctr.add_(1)
        seed = ctr.clone()
    return seed, int(round(keep * 65536)), 1.0 / keep


# Forward pre-scale policy of _ReSpmm: "auto" | "on" | "off" (tools/ab_spmm.py flips it).
# "on": pre * drop(x) is formed once per source row by regnn_row_scale and the aggregation
# gathers the finished rows; "off": the gather scales and masks every edge's row itself.
# "prefix": an aggregation backward whose gradient is known zero past row n (the output head's
# hand-off) gathers only the CSC edges into rows < n ("off": the whole CSC)
# "self": the input projection skips h when the first aggregation's backward can read its
# pre-scaled rows instead (type_project_prescale keep_h=False; "off": h always written)
PRESCALE = {"mode": "auto", "bwd": "auto", "next": "auto", "prefix": "auto", "self": "auto"}


def _use_prescale(x, scale, drop, backward=False):
    """forward: scale = pre (source rows), drop = the fused dropout; backward: scale = post
    (the gradient rows the transposed aggregation gathers)."""
    mode = PRESCALE["bwd" if backward else "mode"]
    if mode == "off" or (scale is None and drop is None):
        return False
    # on / auto: one streaming pass over the rows (2*N*F*s bytes) takes the E*F mask hashes and
    # the E dependent scale lookups out of the gather; measured faster for fp32 and bf16 at
    # F = 64 on mag-10x (tools/ab_spmm.py)
    return True


class _NextLink:
    """Backward hand-off between two chained aggregations y' = post' * (A' x') and y = A(..y'..).

    When the consumer reads y' as its input x unchanged (no op in between and no other consumer),
    the producer's backward needs post' * g' and <g', y'> / post' for g' = d loss / d y' = the
    consumer's gx. The consumer's backward forms both in its epilogue (regnn_spmm_bwd_next) and
    parks them here; the producer's backward takes them only if its incoming gradient IS that gx
    tensor, unmodified (autograd summed nothing into it), and runs its own row pass otherwise.
    The hand-off's last field, when not None, is a row count n such that the gradient is zero on
    rows >= n (the output head's loss rows) and the handed rows >= n are not written: the
    producer's transposed gather must then run over the CSC prefix of edges into rows < n
    (RelGraph.csc_prefix), or not take the hand-off."""

    __slots__ = ("post", "handoff")

    def __init__(self, post):
        self.post = post
        self.handoff = None

    def take(self, gy):
        h, self.handoff = self.handoff, None
        if h is None:
            return None
        gx, version, nx_out, nx_dot, nz = h
        if gy is not gx or gy._version != version:
            return None
        return nx_out, nx_dot, nz


def _drop_args(drop):
    if drop is None:
        return None, 0, 1.0
    return L.ptr(drop[0]), drop[1], drop[2]


class _ReSpmm(torch.autograd.Function):
    """y = post * (A_tab (pre * drop(x))) + bias, A_tab[v,u] = sum over edges u->v of tab[rel_e];
    drop = the optional fused dropout of the gathered rows (regnn_spmm_fwd_dropout)."""

    @staticmethod
    def forward(ctx, x, tab, pre, post, bias, rg, pack, drop=None, prescaled=None, link=None,
                link_in=None, emit=None):
        x = x.contiguous()
        F = x.shape[1]
        y = torch.empty(rg.n_dst, F, dtype=x.dtype, device=x.device)
        t = _flat_table(tab)
        plan_args, part = _plan_args(rg.csr_plan, F, x.device)
        # prescaled: pre * drop(x) already formed by the producer of x (regnn_type_project)
        prescale = prescaled is None and _use_prescale(x, pre, drop)
        src, in_scale = (x, pre) if prescaled is None else (prescaled, None)
        with timed("spmm_fwd", spmm_bytes(rg.E, rg.n_dst, rg.n_src, F, x.element_size(),
                                          "spmm_fwd")):
            if prescale:
                # pre * drop(x) once per source row (regnn_row_scale), then a plain gather
                src, in_scale = torch.empty_like(x), None
                L.call("regnn_row_scale", L.ptr(x), L.ptr(pre), L.ptr(src), x.shape[0], F,
                       L.dtype_code(x), *(_drop_args(drop)), None, None, L.stream())
            args = (L.ptr(rg.csr_ptr), L.ptr(rg.csr_idx),
                    L.ptr(pack.rel_csr if (pack is not None and t is not None) else None),
                    L.ptr(t), None, L.ptr(in_scale), L.ptr(post),
                    L.ptr(None if bias is None else bias.detach().float().contiguous()),
                    L.ptr(src), L.ptr(y), rg.n_dst, F, L.dtype_code(x), *plan_args)
            if emit is not None:
                # the consumer's pre-scaled rows drop'(scale * y) leave from the same epilogue
                nscale, ndrop = emit[0], emit[1]
                xs = torch.empty_like(y)
                gdrop = drop if (drop is not None and not prescale and prescaled is None) else None
                L.call("regnn_spmm_fwd_next", *args, *(_drop_args(gdrop)), L.ptr(nscale),
                       *(_drop_args(ndrop)), L.ptr(xs), L.stream())
                emit[2] = xs
            elif drop is None or prescale or prescaled is not None:
                L.call("regnn_spmm_fwd", *args, L.stream())
            else:
                L.call("regnn_spmm_fwd_dropout", *args, L.ptr(drop[0]), drop[1], drop[2],
                       L.stream())
        del src
        ctx.drop = drop
        ctx.link, ctx.link_in = link, link_in
        ctx.rg, ctx.pack, ctx.tab_shape = rg, pack, None if tab is None else tab.shape
        ctx.same_scale = pre is not None and pre is post and rg.n_src == rg.n_dst
        # x never written (type_project_prescale keep_h=False): the backward reads the gathered
        # rows pre * drop(x) instead (REGNN_SELF_PRESCALED; pre is a positive degree norm)
        ctx.self_pre = getattr(x, "_regnn_unwritten", False)
        if ctx.self_pre:
            if prescaled is None or pre is None or link_in is not None:
                raise RuntimeError("re_spmm: an unwritten input needs its pre-scaled rows")
            x = prescaled
        ctx.save_for_backward(x, y, t, pre, post)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, y, t, pre, post = ctx.saved_tensors
        rg, pack = ctx.rg, ctx.pack
        need_x, need_tab, need_pre, need_post, need_bias = ctx.needs_input_grad[:5]
        gy = gy.contiguous().to(x.dtype)
        F = x.shape[1]
        gx = torch.empty(rg.n_src, F, dtype=x.dtype, device=x.device)
        n_rel = t.numel() if t is not None else 0
        slab = _slab(n_rel, x.device) if (need_tab and t is not None) else None
        node = None
        if ctx.same_scale and (need_pre or need_post):
            node = torch.empty(rg.n_src, dtype=torch.float32, device=x.device)
        elif need_pre:
            node = torch.empty(rg.n_src, dtype=torch.float32, device=x.device)
        # output-side norm gradient <g, y> / post: same-scale node term or d loss / d post
        want_dot = (ctx.same_scale and node is not None) or (not ctx.same_scale and need_post)
        prescale = post is not None and _use_prescale(x, post, None, backward=True)
        src, in_scale, dot = gy, post, None
        drop = ctx.drop
        handed = ctx.link.take(gy) if (prescale and ctx.link is not None) else None
        if handed is not None and handed[2] is not None and handed[2] < rg.n_dst and \
                PRESCALE["prefix"] == "off":
            handed = None          # its rows >= nz are not written: only the prefix may use it
        # the consumer of x (the next aggregation) forms its producer's pre-scaled gradient rows
        nx = ctx.link_in if (need_x and ctx.link_in is not None and
                             ctx.link_in.post.numel() == rg.n_src) else None
        # gradient rows >= nz known zero (hand-off from the output head): gather only the CSC
        # edges into rows < nz; the skipped edges' terms are exact zeros
        pre_g = rg.csc_prefix(handed[2]) if (handed is not None and handed[2] is not None and
                                             PRESCALE["prefix"] != "off") else None
        csc_ptr, csc_idx, csc_plan, E_b = (rg.csc_ptr, rg.csc_idx, rg.csc_plan, rg.E) \
            if pre_g is None else (pre_g.csc_ptr, pre_g.csc_idx, pre_g.csc_plan, pre_g.E)
        rel_csc = None
        if pack is not None and t is not None:
            rel_csc = pack.rel_csc if pre_g is None else pack.rel_csc_prefix(pre_g)
        plan_args, part = _plan_args(csc_plan, F, x.device)
        with timed("spmm_bwd", spmm_bytes(E_b, rg.n_dst, rg.n_src, F, x.element_size(),
                                          "spmm_bwd")):
            if handed is not None:
                # post * g and <g, y> / post came from the consumer's backward epilogue
                src, in_scale = handed[0], None
                dot = handed[1] if want_dot else None
            elif prescale:
                # post * g once per destination row (regnn_row_scale), with <g, y> / post formed
                # in the same pass; the transposed gather then reads finished rows
                src, in_scale = torch.empty_like(gy), None
                dot = torch.empty(rg.n_dst, dtype=torch.float32, device=x.device) if want_dot \
                    else None
                L.call("regnn_row_scale", L.ptr(gy), L.ptr(post), L.ptr(src), rg.n_dst, F,
                       L.dtype_code(x), None, 0, 1.0, L.ptr(y if want_dot else None), L.ptr(dot),
                       L.stream())
            args = (L.ptr(csc_ptr), L.ptr(csc_idx), L.ptr(rel_csc),
                    L.ptr(t), None, L.ptr(in_scale), L.ptr(pre), L.ptr(src), L.ptr(x),
                    L.ptr(y if ctx.same_scale and node is not None and not prescale else None),
                    L.ptr(gx), L.ptr(slab), n_rel, None, L.ptr(node), rg.n_src, F,
                    L.dtype_code(x) | (L.SELF_PRESCALED if ctx.self_pre else 0), *plan_args)
            if nx is not None:
                nx_out = torch.empty_like(gx)
                nx_dot = torch.empty(rg.n_src, dtype=torch.float32, device=x.device)
                L.call("regnn_spmm_bwd_next", *args, *(_drop_args(drop)),
                       L.ptr(nx.post), L.ptr(nx_out), L.ptr(nx_dot), L.stream())
                nx.handoff = (gx, gx._version, nx_out, nx_dot, None)
            elif drop is None:
                L.call("regnn_spmm_bwd", *args, L.stream())
            else:
                L.call("regnn_spmm_bwd_dropout", *args, L.ptr(drop[0]), drop[1], drop[2],
                       L.stream())
            if prescale and ctx.same_scale and node is not None:
                node.add_(dot)
        del src
        g_tab = _reduce(slab, n_rel).view(ctx.tab_shape) if slab is not None else None
        g_pre = g_post = None
        if ctx.same_scale:
            g_pre = node
        else:
            if need_pre:
                g_pre = node
            if need_post:
                if dot is not None:
                    g_post = dot
                else:
                    yf, gf = y.float(), gy.float()
                    g_post = (gf * yf).sum(1) / post
        g_bias = gy.float().sum(0) if need_bias else None
        return (gx if need_x else None), g_tab, g_pre, g_post, g_bias, None, None, None, None, \
            None, None, None


def re_spmm(rg, x, tab=None, pack=None, pre=None, post=None, bias=None, dropout=0.0,
            drop_seed=None, prescaled=None, emit=None):
    """y[v] = post[v] * sum_{e: u->v} tab[rel_e] * pre[u] * drop(x)[u] + bias  (HIP).

    dropout: probability of an nn.Dropout applied to x in front of the aggregation; fused into
    the gather for 256-byte rows (no dropped copy, no mask tensor), a torch dropout otherwise.
    The bias is fused into the kernel epilogue unless the backward needs the pre-bias output
    (differentiable post-scale: the node-norm gradient reads <g, y> / post).

    prescaled: pre * drop(x) formed by x's producer (type_project_prescale, same pre and
    drop_seed); the forward gathers it directly, the backward is unchanged.

    emit: (scale, drop) of a consumer aggregation that reads y as its input (drop a
    drop_request or None): returns (y, xs) with xs = drop(scale * y) from the same epilogue
    (regnn_spmm_fwd_next), the consumer's `prescaled`; xs is None where the epilogue cannot form
    it (bias added outside the op), and the consumer then runs its own row pass."""
    drop = None
    if dropout:
        if dropout < 1.0 and dropout_fusable(x):
            drop = drop_request(dropout, x.device, drop_seed)
        else:
            if prescaled is not None:
                raise ValueError("prescaled input with an unfusable dropout")
            x = torch.nn.functional.dropout(x, dropout, training=True)
    # x produced by another aggregation, read as is: this op's backward hands the producer its
    # pre-scaled gradient rows (_NextLink, regnn_spmm_bwd_next)
    link_in = getattr(x, "_regnn_link", None)
    if link_in is not None and (not x.is_cuda or not dropout_fusable(x)):
        link_in = None
    if bias is not None and post is not None and post.requires_grad:
        y = _ReSpmm.apply(x, tab, pre, post, None, rg, pack, drop, prescaled, None,
                          link_in) + bias
        return y if emit is None else (y, None)
    link = None
    if post is not None and x.is_cuda and PRESCALE["next"] != "off" and \
            PRESCALE["bwd"] != "off":
        link = _NextLink(post.detach())
    holder = None
    if emit is not None and PRESCALE["next"] != "off" and x.is_cuda and \
            (emit[1] is None or dropout_fusable(x)):
        holder = [emit[0].detach().float().contiguous(), emit[1], None]
    y = _ReSpmm.apply(x, tab, pre, post, bias, rg, pack, drop, prescaled, link, link_in, holder)
    if link is not None:
        y._regnn_link = link
    if emit is None:
        return y
    return y, (None if holder is None else holder[2])


class _TypeProjPre(torch.autograd.Function):
    """h = cat_t(x_t W_t^T + b_t) and xs = scale * drop(h) in one HIP pass per node type
    (regnn_type_project); xs is a non-differentiable side output for the aggregation's gather,
    d h flows to W_t / b_t as in nets._TypeProjFn."""

    @staticmethod
    def forward(ctx, n, scale, drop, keep_h, *args):
        xs_in, Ws, bs = args[:n], args[n:2 * n], args[2 * n:]
        rows = [x.shape[0] for x in xs_in]
        dev, dt = xs_in[0].device, xs_in[0].dtype
        F = Ws[0].shape[0]
        h = torch.empty(sum(rows), F, dtype=dt, device=dev)
        xs = torch.empty_like(h)
        seed, keep16, dscale = (None, 0, 1.0) if drop is None else (L.ptr(drop[0]), drop[1],
                                                                    drop[2])
        sc = None if scale is None else scale.detach().float().contiguous()
        o = 0
        with timed("type_project", sum(x.numel() * x.element_size() for x in xs_in)
                   + (2 if keep_h else 1) * h.numel() * h.element_size()):
            for x, W, b, r in zip(xs_in, Ws, bs, rows):
                x = x.contiguous()
                L.call("regnn_type_project", L.ptr(x), r, x.shape[1], F, L.dtype_code(x),
                       L.ptr(W.detach().float().contiguous()),
                       L.ptr(b.detach().float().contiguous()), L.ptr(sc), seed, keep16, dscale,
                       o, L.ptr(h) if keep_h else None, L.ptr(xs), L.stream())
                o += r
        ctx.n, ctx.rows = n, rows
        ctx.save_for_backward(*xs_in, *Ws)
        ctx.mark_non_differentiable(xs)
        ctx.set_materialize_grads(False)      # no N x F zero gradient for the side output xs
        return h, xs

    @staticmethod
    def backward(ctx, g, _gxs):
        n = ctx.n
        if g is None:
            return (None,) * (4 + 3 * n)
        saved = ctx.saved_tensors
        xs_in, Ws = saved[:n], saved[n:]
        g = g.contiguous()
        gx, gW, gb = [None] * n, [None] * n, [None] * n
        o = 0
        for t, r in enumerate(ctx.rows):
            gt = g[o:o + r]
            o += r
            if ctx.needs_input_grad[4 + t]:
                gx[t] = gt @ Ws[t].to(gt.dtype)
            if ctx.needs_input_grad[4 + n + t] or ctx.needs_input_grad[4 + 2 * n + t]:
                w_, b_ = linear_wgrad(gt, xs_in[t])
                gW[t] = w_.to(Ws[t].dtype)
                gb[t] = b_.to(Ws[t].dtype)
        return (None, None, None, None, *gx, *gW, *gb)


def type_project_fusable(fcs, feats, width=64):
    """regnn_type_project's shapes: every type a biased Linear to `width` = 64 from <= 256
    features, one storage dtype (fp32 / bf16) on the device."""
    return (width == 64 and len(fcs) == len(feats) > 0
            and all(fc.bias is not None and fc.weight.shape[0] == 64 and fc.weight.shape[1] <= 256
                    for fc in fcs)
            and all(f.is_cuda and f.dim() == 2 and f.dtype == feats[0].dtype for f in feats)
            and feats[0].dtype in (torch.float32, torch.bfloat16))


def type_project_prescale(fcs, feats, scale, drop, keep_h=True):
    """(h, xs): the concatenated per-type projections and scale * drop(h) (model/REGCN.py:31-35
    + the first layer's pre-scale, layer/REGraphConv.py:56,73-76) from one HIP pass per type.

    keep_h=False: h is not written (an allocated, unwritten tensor marked `_regnn_unwritten`);
    only an aggregation that gathers xs (re_spmm prescaled=xs) may take it, and its backward
    then reads xs for the terms that need h (REGNN_SELF_PRESCALED)."""
    keep_h = keep_h or PRESCALE["self"] == "off"
    h, xs = _TypeProjPre.apply(len(fcs), scale, drop, keep_h, *feats,
                               *[fc.weight for fc in fcs], *[fc.bias for fc in fcs])
    if not keep_h:
        h._regnn_unwritten = True
    return h, xs


def re_spmm_fused(rg, x, tab=None, pack=None, post=None, bias=None, residual=None, ln=None,
                  relu=False):
    """forward-only y = act(LN(post * (A_tab x) + bias + residual)) in one HIP pass
    (regnn_spmm_fwd_fused; the mag REGCNConv tail at inference, mag/regnn_layers.py:129-135 +
    mag/regnn_ns.py:362). ln = (weight, bias, eps) of a LayerNorm, or None."""
    if torch.is_grad_enabled() and any(t is not None and t.requires_grad
                                       for t in (x, tab, post, bias, residual)):
        raise RuntimeError("re_spmm_fused is forward-only (use it under torch.no_grad())")
    x = x.contiguous()
    F = x.shape[1]
    y = torch.empty(rg.n_dst, F, dtype=x.dtype, device=x.device)
    t = _flat_table(tab)
    plan_args, part = _plan_args(rg.csr_plan, F, x.device)
    epi = (1 if ln is not None else 0) | (2 if relu else 0)
    lw = lb = None
    eps = 0.0
    if ln is not None:
        lw, lb, eps = ln
        lw = None if lw is None else lw.detach().float().contiguous()
        lb = None if lb is None else lb.detach().float().contiguous()
    res = None if residual is None else residual.contiguous().to(x.dtype)
    with timed("spmm_fwd", spmm_bytes(rg.E, rg.n_dst, rg.n_src, F, x.element_size(),
                                      "spmm_fwd")):
        L.call("regnn_spmm_fwd_fused", L.ptr(rg.csr_ptr), L.ptr(rg.csr_idx),
               L.ptr(pack.rel_csr if (pack is not None and t is not None) else None),
               L.ptr(t), None, None, L.ptr(post),
               L.ptr(None if bias is None else bias.detach().float().contiguous()),
               L.ptr(x), L.ptr(y), rg.n_dst, F, L.dtype_code(x), *plan_args, L.ptr(res),
               L.ptr(lw), L.ptr(lb), float(eps), epi, L.stream())
    return y


# ---------------------------------------------------------------------------------------------
_NO_PLAN = (0, 0, None, 0, None, None, 0, None, None, 0, None)


_CSC_WIDTHS = (64, 128, 256, 512, 1024, 2048)   # regnn_ns_spmm_bwd_csc's F = 4 LPR VPL
# "auto": a sampled block carrying its transposed index differentiates by the CSC gather; "off":
# the atomic scatter (tests compare the two)
NS_CSC = {"mode": "auto"}
# "on": the CSC gather's hub rows in chunks over the grid (regnn_ns_spmm_bwd_csc hub_work);
# "off": a workgroup per hub row
NS_CSC_CHUNKED = {"mode": os.environ.get("REGNN_NS_CSC_CHUNKED", "on")}
# workgroups of regnn_ns_spmm_bwd_csc with relation dots (one relation-slab row each; 0:
# L.slab_rows() = 4096). 1024: each row group takes ~3 of a 13 312-row block's rows instead of
# one, and the slab reduce reads a quarter of the rows -- hidden 512, mag-10x: 416.2-418.7 against
# 424.5-425.4 us per step (512: 418.3-420.3, 2048: 420.8-420.9)
CSC_BWD_ROWS = {"n": int(os.environ.get("REGNN_NS_CSC_BWD_ROWS", "1024"))}
# workgroups of regnn_ns_slot_agg_bwd (one relation-slab row each; 0: a row per 8 of the block's
# capacity rows, at most L.slab_rows(): 1664 at mag-10x, 414.2-414.6 us per step at hidden 512
# against 417.6 with 1024 and 419.1-419.7 with 512)
SLOT_BWD_ROWS = {"n": int(os.environ.get("REGNN_NS_SLOT_BWD_ROWS", "0"))}
# include/regnn_hip.h REGNN_CSC_LONG_INTS (the sampler's csc_long with the hub piece table)
CSC_LONG_INTS = ((32768 // 17 + 1 + 2) + 3) // 4 * 4 + 4 * (32768 // 1024 + 32768 // 17 + 1)  # PIECE 1024
_HUB_WORK = {}


def _hub_work(F, device):
    key = (F, device)
    if key not in _HUB_WORK:
        _HUB_WORK[key] = torch.empty(int(L._so.regnn_ns_csc_hub_work_floats(F)),
                                     dtype=torch.float32, device=device)
    return _HUB_WORK[key]


class _NsSpmm(torch.autograd.Function):
    """y[v] = inv[v] * sum_{e in row v} tab[rel_e] * x[idx_e] + bias over a sampled block
    (regnn_hip.ns.NSBlock: rows <= fan-out + 1, no long-row plan, no host sizes)."""

    @staticmethod
    def forward(ctx, x, tab, bias, blk):
        x = x.contiguous()
        if x.dtype != torch.float32:
            raise TypeError("ns_spmm: the sampled-block aggregation runs on fp32 rows")
        F = x.shape[1]
        y = torch.empty(blk.n_dst, F, dtype=x.dtype, device=x.device)
        t = _flat_table(tab)
        strided = getattr(blk, "strided_rows", None)
        if strided is not None:
            # the sampler wrote this block in the strided layout: row i at slots i S ..
            cnt, S = strided
            b = None if bias is None else bias.detach().float().contiguous()
            with timed("ns_spmm_fwd", spmm_bytes(blk.E, blk.n_dst, blk.n_src, F, 4, "spmm_fwd")):
                L.call("regnn_ns_spmm_strided_fwd", L.ptr(blk.live_rows), L.ptr(cnt), S,
                       L.ptr(blk.csr_idx), L.ptr(blk.rel if t is not None else None), L.ptr(t),
                       L.ptr(blk.inv), L.ptr(b), L.ptr(x), L.ptr(y), blk.n_dst, F, L.stream())
            ctx.blk, ctx.tab_shape = blk, None if tab is None else tab.shape
            ctx.save_for_backward(x, t)
            return y
        with timed("ns_spmm_fwd", spmm_bytes(blk.E, blk.n_dst, blk.n_src, F, 4, "spmm_fwd")):
            L.call("regnn_spmm_fwd", L.ptr(blk.csr_ptr), L.ptr(blk.csr_idx),
                   L.ptr(blk.rel if t is not None else None), L.ptr(t), None, None,
                   L.ptr(blk.inv), L.ptr(None if bias is None else bias.detach().float().contiguous()),
                   L.ptr(x), L.ptr(y), blk.n_dst, F, L.F32_CODE, *_NO_PLAN, L.stream())
        ctx.blk, ctx.tab_shape = blk, None if tab is None else tab.shape
        ctx.save_for_backward(x, t)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, t = ctx.saved_tensors
        blk = ctx.blk
        need_x, need_tab, _, = ctx.needs_input_grad[:3]
        gy = gy.contiguous().float()
        F = x.shape[1]
        n_rel = t.numel() if t is not None else 0
        csc = getattr(blk, "csc", None)
        if csc is not None and NS_CSC["mode"] != "off" and F in _CSC_WIDTHS and \
                x.shape[0] <= blk.csc_cap:
            # a gather over the sampler's transposed index: every row written once, no atomics
            cptr, cent, clong, sizes, size_idx = csc
            gx = torch.empty_like(x)
            # the launch's workgroups = its relation-slab rows (grid-stride over the rows and the
            # hub chunks); REGNN_NS_CSC_BWD_ROWS caps them (A/B)
            rows = min(L.slab_rows(), CSC_BWD_ROWS["n"]) if CSC_BWD_ROWS["n"] > 0 else L.slab_rows()
            slab = (torch.empty(rows, n_rel, dtype=torch.float32, device=x.device)
                    if (need_tab and t is not None) else None)
            # the hub rows chunked over the grid (a workgroup per 8 entries per row group
            # instead of per hub row: ~500-entry hubs at fan-out 25 dominated at F = 512)
            hub = None
            if NS_CSC_CHUNKED["mode"] != "off" and clong.numel() >= CSC_LONG_INTS:
                hub = _hub_work(F, x.device)
            with timed("ns_spmm_bwd", spmm_bytes(blk.E, blk.n_dst, blk.n_src, F, 4, "spmm_bwd")):
                L.call("regnn_ns_spmm_bwd_csc", L.ptr(cptr), L.ptr(cent), L.ptr(clong), L.ptr(t),
                       L.ptr(blk.inv),
                       L.ptr(gy), L.ptr(x), L.ptr(gx), L.ptr(slab), n_rel, L.ptr(sizes), size_idx,
                       x.shape[0], F, rows, L.ptr(hub), L.stream())
            g_tab = _reduce(slab, n_rel).view(ctx.tab_shape) if slab is not None else None
            g_bias = gy.sum(0) if ctx.needs_input_grad[2] else None
            return (gx if need_x else None), g_tab, g_bias, None
        if getattr(blk, "strided_rows", None) is not None:
            raise RuntimeError("ns_spmm: a strided block differentiates through its transposed "
                               "index only (NS_CSC on, F in %s)" % (_CSC_WIDTHS,))
        gx = torch.zeros_like(x)
        slab = _slab(n_rel, x.device) if (need_tab and t is not None) else None
        with timed("ns_spmm_bwd", spmm_bytes(blk.E, blk.n_dst, blk.n_src, F, 4, "spmm_bwd")):
            L.call("regnn_ns_spmm_bwd", L.ptr(blk.csr_ptr), L.ptr(blk.csr_idx),
                   L.ptr(blk.rel if t is not None else None), L.ptr(t), L.ptr(blk.inv), L.ptr(gy),
                   L.ptr(x), L.ptr(gx), L.ptr(slab), n_rel, blk.n_dst, F, L.stream())
        g_tab = _reduce(slab, n_rel).view(ctx.tab_shape) if slab is not None else None
        g_bias = gy.sum(0) if ctx.needs_input_grad[2] else None
        return (gx if need_x else None), g_tab, g_bias, None


def ns_spmm(blk, x, tab=None, bias=None):
    """mean aggregation of a sampled block with the relation table and the bias fused
    (mag/regnn_layers.py:110-148: ew = LeakyReLU(rw)[type], propagate aggr='mean', update +bias).
    x holds the block's source rows (>= blk.n_src rows; rows past the sampled ones unread)."""
    return _NsSpmm.apply(x, tab, bias, blk)



class _NsTypedAgg(torch.autograd.Function):
    """S[v, t] = sum_{e in v, type(src) = t} tab[rel_e] x_src (raw input rows read through n_id /
    node type / local row), w[v, t] = sum of the same tab[rel_e] (regnn_ns_typed_agg), returned
    as one [n_dst, T K + T] tensor [S | w] (ext) or as (S [n_dst, T, K], w [n_dst, T]); backward:
    the relation-table gradient only (the input tables are data, feats_type 3)."""

    @staticmethod
    def forward(ctx, tab, blk, n_id, tables, node_type, local_idx, ext):
        T, K = len(tables), int(tables[0].shape[1])
        dev = tables[0].device
        if ext:
            # row stride T K + Tp, Tp = T rounded up to 4 (the kernels take 16-byte aligned
            # rows); the Tp - T pad columns are zeros, so a GEMM against [W_c; b_c; 0] is exact
            Tp = _ext_pad(T)
            out = torch.empty(blk.n_dst, T * K + Tp, dtype=torch.float32, device=dev)
            if Tp != T:
                out[:, T * K + T:].zero_()
            S_ptr, w_ptr, lds, ldw = L.ptr(out), L.ptr(out) + 4 * T * K, T * K + Tp, T * K + Tp
        else:
            S = torch.empty(blk.n_dst, T, K, dtype=torch.float32, device=dev)
            w = torch.empty(blk.n_dst, T, dtype=torch.float32, device=dev)
            S_ptr, w_ptr, lds, ldw = L.ptr(S), L.ptr(w), T * K, T
        t = tab.detach().float().contiguous()
        meta = getattr(blk, "edge_meta", None)
        if meta is not None:
            # a meta-only hop: each edge's source type / table row straight from the sampler
            n_id = node_type = local_idx = None
            e_type, e_off = meta
        else:
            n_id = _i32(n_id)
            node_type = _cached_cast(node_type, torch.int32)
            local_idx = _cached_cast(local_idx, torch.int64)
            e_type = e_off = None
        arr = _ptr_array([L.ptr(x) for x in tables])
        with timed("ns_typed_agg", blk.E * (4 * K + 13) + blk.n_dst * (T * 4 * K + 4 * T + 8)):
            L.call("regnn_ns_typed_agg", L.ptr(blk.csr_ptr), L.ptr(blk.csr_idx), L.ptr(blk.rel),
                   L.ptr(t), L.ptr(n_id), L.ptr(node_type), L.ptr(local_idx), L.ptr(e_type),
                   L.ptr(e_off), arr, T, K, blk.n_dst, S_ptr, w_ptr, lds, ldw, L.stream())
        ctx.blk, ctx.tables, ctx.idx = blk, tables, (n_id, node_type, local_idx, e_type, e_off)
        ctx.n_rel, ctx.tab_shape, ctx.ext = t.numel(), tab.shape, bool(ext)
        return out if ext else (S, w)

    @staticmethod
    def backward(ctx, *grads):
        if not ctx.needs_input_grad[0]:
            return (None,) * 7
        blk, tables = ctx.blk, ctx.tables
        n_id, node_type, local_idx, e_type, e_off = ctx.idx
        T, K = len(tables), int(tables[0].shape[1])
        dev = tables[0].device
        if ctx.ext:
            g = grads[0]
            Tp = _ext_pad(T)
            g = (torch.zeros(blk.n_dst, T * K + Tp, device=dev) if g is None
                 else g.contiguous().float())
            gS_ptr, gw_ptr, lds, ldw = L.ptr(g), L.ptr(g) + 4 * T * K, T * K + Tp, T * K + Tp
        else:
            gS, gw = grads
            gS = (torch.zeros(blk.n_dst, T, K, device=dev) if gS is None
                  else gS.contiguous().float())
            gw = torch.zeros(blk.n_dst, T, device=dev) if gw is None else gw.contiguous().float()
            gS_ptr, gw_ptr, lds, ldw = L.ptr(gS), L.ptr(gw), T * K, T
        rows = L.slab_rows()
        slab = torch.empty(rows, ctx.n_rel, dtype=torch.float32, device=dev)
        with timed("ns_typed_agg_bwd", blk.E * (4 * K + 13) + blk.n_dst * (T * 4 * K + 4 * T + 8)):
            L.call("regnn_ns_typed_agg_bwd", L.ptr(blk.csr_ptr), L.ptr(blk.csr_idx),
                   L.ptr(blk.rel), L.ptr(n_id), L.ptr(node_type), L.ptr(local_idx),
                   L.ptr(e_type), L.ptr(e_off),
                   _ptr_array([L.ptr(x) for x in tables]), T, K, blk.n_dst, gS_ptr, gw_ptr,
                   lds, ldw, L.ptr(slab), ctx.n_rel, rows, L.stream())
        return _reduce(slab, ctx.n_rel).view(ctx.tab_shape), None, None, None, None, None, None


class _NsSlotAgg(torch.autograd.Function):
    """[S | w | 0] of regnn_ns_typed_agg (ext) from the sampler's per-type input sums (relation
    slots; regnn_ns_slot_agg): pre = the slot's U [cap, T, K], counts [cap, T], self rows [cap, K]
    and slot relations [cap, T + 1] the outer hop's sums launch wrote; backward: the relation
    table's gradient (regnn_ns_slot_agg_bwd + the fixed-order slab reduce)."""

    @staticmethod
    def forward(ctx, tab, blk, pre, n_et):
        U, cnt, xself, urel = pre
        cap, T, K = U.shape
        Tp = _ext_pad(T)
        ld = T * K + Tp
        out = torch.empty(cap, ld, dtype=torch.float32, device=U.device)
        t = tab.detach().float().contiguous()
        with timed("ns_slot_agg"):
            L.call("regnn_ns_slot_agg", L.ptr(blk.live_rows), 0, L.ptr(U), L.ptr(cnt),
                   L.ptr(xself), L.ptr(urel), L.ptr(t), int(n_et), T, K, cap, L.ptr(out), ld,
                   L.stream())
        ctx.blk, ctx.pre, ctx.n_et = blk, pre, int(n_et)
        ctx.n_rel, ctx.tab_shape = t.numel(), tab.shape
        return out

    @staticmethod
    def backward(ctx, g):
        if not ctx.needs_input_grad[0]:
            return None, None, None, None
        U, cnt, xself, urel = ctx.pre
        cap, T, K = U.shape
        g = g.contiguous().float()
        rows = int(min(L.slab_rows(), max(1, -(-cap // 8))))   # 8 row groups per block
        if SLOT_BWD_ROWS["n"] > 0:
            rows = min(rows, SLOT_BWD_ROWS["n"])
        slab = torch.empty(rows, ctx.n_rel, dtype=torch.float32, device=U.device)
        with timed("ns_slot_agg_bwd"):
            L.call("regnn_ns_slot_agg_bwd", L.ptr(ctx.blk.live_rows), 0, L.ptr(U), L.ptr(cnt),
                   L.ptr(xself), L.ptr(urel), L.ptr(g), g.stride(0), ctx.n_et, T, K, L.ptr(slab),
                   ctx.n_rel, rows, L.stream())
        return _reduce(slab, ctx.n_rel).view(ctx.tab_shape), None, None, None


def ns_slot_agg(blk, tab, n_et):
    """ns_typed_agg(..., ext=True) for a block whose sampler formed layer 0's per-type input sums
    (blk.pre_sums: relation slots, regnn_ns_hop_typed_sums): the same [S | w | 0] operand from one
    read of contiguous sums per row; differentiable in tab."""
    return _NsSlotAgg.apply(tab, blk, blk.pre_sums, int(n_et))


_CAST_CACHE = {}


def _cached_cast(t, dtype):
    """t as a contiguous `dtype` tensor, converted once per (storage, version): the per-node
    tables (node type, local row) are graph-sized and constant across steps."""
    if t.dtype == dtype and t.is_contiguous():
        return t
    key = (t.data_ptr(), t.numel(), t.dtype, dtype, t.device)
    hit = _CAST_CACHE.get(key)
    if hit is not None and hit[0] is t and hit[1] == t._version:
        return hit[2]
    out = t.to(dtype).contiguous()
    if len(_CAST_CACHE) > 16:
        _CAST_CACHE.clear()
    _CAST_CACHE[key] = (t, t._version, out)
    return out


def _ext_pad(T):
    """columns of w in ns_typed_agg's ext rows: T rounded up to a multiple of 4."""
    return (int(T) + 3) // 4 * 4


def ns_typed_agg(blk, tab, n_id, tables, node_type, local_idx, ext=False):
    """layer 0's sampled-block aggregation of the RAW input rows per source node type (the NS
    REGNN's group_input Linear and first conv weight moved after the mean by linearity,
    mag/regnn_ns.py:300-326 + mag/regnn_layers.py:101-148): returns S [n_dst, T, K] and the
    per-type weight sums w [n_dst, T], or with ext one [n_dst, T K + Tp] tensor [S | w | 0]
    (Tp = T rounded up to 4, zero pad columns: the projection's single GEMM operand against
    [W_c; b_c; 0]); differentiable in tab."""
    return _NsTypedAgg.apply(tab, blk, n_id, tables, node_type, local_idx, bool(ext))


def ns_typed_agg_ok(tables):
    """regnn_ns_typed_agg's operand contract: 1..8 fp32 contiguous device tables of one width
    64 or 128."""
    if not tables or len(tables) > 8 or any(t is None for t in tables):
        return False
    K = tables[0].shape[1] if tables[0].dim() == 2 else -1
    return K in (64, 128) and all(
        t.is_cuda and t.dtype == torch.float32 and t.dim() == 2 and t.shape[1] == K and
        t.is_contiguous() and t.data_ptr() % 16 == 0 for t in tables)


class _RelTab(torch.autograd.Function):
    """tab = leaky_relu(alpha rw, slope) in one launch, its backward in one (regnn_rel_tab)."""

    @staticmethod
    def forward(ctx, rw, alpha, slope):
        rw = rw.contiguous()
        out = torch.empty_like(rw)
        L.call("regnn_rel_tab", L.ptr(rw), None, rw.numel(), float(alpha), float(slope),
               L.ptr(out), L.stream())
        ctx.save_for_backward(rw)
        ctx.alpha, ctx.slope = alpha, slope
        return out

    @staticmethod
    def backward(ctx, g):
        (rw,) = ctx.saved_tensors
        g = g.contiguous()
        out = torch.empty_like(rw)
        L.call("regnn_rel_tab", L.ptr(rw), L.ptr(g), rw.numel(), float(ctx.alpha),
               float(ctx.slope), L.ptr(out), L.stream())
        return out, None, None


class _RelTabs(torch.autograd.Function):
    """every layer's relation table in one launch, their backward in one (regnn_rel_tabs)."""

    @staticmethod
    def forward(ctx, alpha, slope, *rws):
        rws = [r.contiguous() for r in rws]
        outs = [torch.empty_like(r) for r in rws]
        n = (ctypes.c_int32 * len(rws))(*[r.numel() for r in rws])
        L.call("regnn_rel_tabs", _ptr_array([L.ptr(r) for r in rws]), None,
               _ptr_array([L.ptr(o) for o in outs]), n, len(rws), float(alpha), float(slope),
               L.stream())
        ctx.save_for_backward(*rws)
        ctx.alpha, ctx.slope = alpha, slope
        return tuple(outs)

    @staticmethod
    def backward(ctx, *gs):
        rws = ctx.saved_tensors
        gs = [torch.zeros_like(r) if g is None else g.contiguous() for r, g in zip(rws, gs)]
        outs = [torch.empty_like(r) for r in rws]
        n = (ctypes.c_int32 * len(rws))(*[r.numel() for r in rws])
        L.call("regnn_rel_tabs", _ptr_array([L.ptr(r) for r in rws]),
               _ptr_array([L.ptr(g) for g in gs]), _ptr_array([L.ptr(o) for o in outs]), n,
               len(rws), float(ctx.alpha), float(ctx.slope), L.stream())
        return (None, None) + tuple(outs)


def rel_tabs(rws, alpha, slope=0.01):
    """[leaky_relu(alpha * rw, slope) for rw in rws] (<= 4 fp32 device tensors) in one launch
    forward and one backward."""
    if not (1 <= len(rws) <= 4 and all(r.is_cuda and r.dtype == torch.float32 for r in rws)):
        raise ValueError("rel_tabs: 1..4 fp32 device tensors")
    return list(_RelTabs.apply(alpha, slope, *rws))


def rel_tab(rw, alpha, slope=0.01):
    """leaky_relu(alpha * rw, slope) (mag/regnn_layers.py:110-111): the relation table of an
    fp32 device relation_weight in one launch instead of a multiply and an activation (and two
    in the backward)."""
    if not (rw.is_cuda and rw.dtype == torch.float32):
        raise ValueError("rel_tab: an fp32 device tensor")
    return _RelTab.apply(rw, alpha, slope)


class _SoftmaxXent(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z, y, ignore):
        z = z.contiguous().float()
        y = y.contiguous()
        B, C = z.shape
        lse = torch.empty(B, dtype=torch.float32, device=z.device)
        rowloss = torch.empty(2 * B, dtype=torch.float32, device=z.device)
        out = torch.empty(2, dtype=torch.float32, device=z.device)
        L.call("regnn_softmax_xent_fwd", L.ptr(z), L.ptr(y), B, C, int(ignore), L.ptr(lse),
               L.ptr(rowloss), L.ptr(out), L.stream())
        ctx.save_for_backward(z, y, lse, out)
        ctx.ignore = int(ignore)
        return out[0]

    @staticmethod
    def backward(ctx, g):
        z, y, lse, out = ctx.saved_tensors
        B, C = z.shape
        gz = torch.empty_like(z)
        g = g.reshape(1).contiguous().float()
        L.call("regnn_softmax_xent_bwd", L.ptr(z), L.ptr(y), L.ptr(lse), L.ptr(out), L.ptr(g), B,
               C, ctx.ignore, L.ptr(gz), L.stream())
        return gz, None, None


def softmax_xent(z, y, ignore=-100):
    """nll_loss(log_softmax(z), y, ignore_index) (mean over the non-ignored rows) from fp32 logits
    in one launch forward and one backward (regnn_softmax_xent_*); y int64."""
    if not (z.is_cuda and z.dim() == 2 and y.dtype == torch.int64):
        raise ValueError("softmax_xent: [B, C] device logits, int64 labels")
    return _SoftmaxXent.apply(z, y, ignore)


class _NsLinXent(torch.autograd.Function):
    """out_lin + log_softmax + nll over a capacity-sized sampled batch: z = x W^T + b on hipBLASLt,
    then the labels, the per-row loss and the fixed-order mean in one launch
    (regnn_ns_xent_fwd); backward: gz and out_lin's bias gradient in one launch
    (regnn_xent_bwd_colsum), gx = gz W and gW = gz^T x on hipBLASLt."""

    @staticmethod
    def forward(ctx, x, w, b, n_id, sizes, labels, ticket, ignore):
        z = torch.addmm(b, x, w.t())
        B, C = z.shape
        y = torch.empty(B, dtype=torch.int64, device=z.device)
        lse = torch.empty(B, dtype=torch.float32, device=z.device)
        rowloss = torch.empty(2 * B, dtype=torch.float32, device=z.device)
        out = torch.empty(2, dtype=torch.float32, device=z.device)
        L.call("regnn_ns_xent_fwd", L.ptr(z), L.ptr(n_id), L.ptr(sizes), L.ptr(labels), B, C,
               int(ignore), L.ptr(y), L.ptr(lse), L.ptr(rowloss), L.ptr(out), L.ptr(ticket),
               L.stream())
        ctx.save_for_backward(x, w, z, y, lse, out)
        ctx.ignore = int(ignore)
        return out[0]

    @staticmethod
    def backward(ctx, g):
        x, w, z, y, lse, out = ctx.saved_tensors
        B, C = z.shape
        gz = torch.empty_like(z)
        gb = torch.empty(C, dtype=torch.float32, device=z.device)
        g = g.reshape(1).contiguous().float()
        L.call("regnn_xent_bwd_colsum", L.ptr(z), L.ptr(y), L.ptr(lse), L.ptr(out), L.ptr(g), B, C,
               ctx.ignore, L.ptr(gz), L.ptr(gb), L.stream())
        gx = gz @ w if ctx.needs_input_grad[0] else None
        gw = gz.t() @ x if ctx.needs_input_grad[1] else None
        return gx, gw, gb, None, None, None, None, None


def ns_lin_xent(x, w, b, n_id, sizes, labels, ticket, ignore=-100):
    """nll_loss(log_softmax(x W^T + b), y) with y[i] = labels[n_id[i]] for i < sizes[0] and
    `ignore` past the batch's live targets (mag/regnn_ns.py:346,404-405 over a capacity-sized
    batch): 3 launches forward (GEMM, loss) and 3 backward (loss + bias gradient, two GEMMs).
    x [B, K] fp32, w [C, K], b [C]; n_id / sizes int32, labels int64 device tensors; ticket: one
    zeroed int32 device word, reused call after call."""
    if not (x.is_cuda and x.dim() == 2 and x.dtype == torch.float32 and w.dtype == torch.float32
            and b is not None and n_id.dtype == torch.int32 and labels.dtype == torch.int64 and
            ticket.dtype == torch.int32 and ticket.numel() >= 1):
        raise ValueError("ns_lin_xent: fp32 [B, K] rows / weight / bias, int32 n_id, int64 "
                         "labels, an int32 ticket")
    return _NsLinXent.apply(x.contiguous(), w, b, n_id, sizes, labels.contiguous(), ticket, ignore)


def ns_labels(n_id, sizes, labels, B, ignore=-100):
    """y[i] = labels[n_id[i]] for the batch's live targets i < sizes[0], else `ignore`
    (mag/regnn_ns.py:404 over a capacity-sized batch) in one launch; n_id int32, labels int64."""
    if n_id.dtype != torch.int32 or labels.dtype != torch.int64 or not n_id.is_cuda:
        raise ValueError("ns_labels: int32 n_id, int64 labels, device tensors")
    y = torch.empty(B, dtype=torch.int64, device=n_id.device)
    L.call("regnn_ns_labels", L.ptr(n_id), L.ptr(sizes), L.ptr(labels.contiguous()), int(B),
           int(ignore), L.ptr(y), L.stream())
    return y


# ---------------------------------------------------------------------------------------------
class _EdgeSpmm(torch.autograd.Function):
    """y[v] = sum_{e: u->v} ew[e] * x[u]; ew per edge in the caller's edge order."""

    @staticmethod
    def forward(ctx, x, ew, rg):
        x = x.contiguous()
        F = x.shape[1]
        ewf = ew.detach().reshape(-1).float()
        w_csr = ewf[rg.csr_eid].contiguous()
        y = torch.empty(rg.n_dst, F, dtype=x.dtype, device=x.device)
        plan_args, part = _plan_args(rg.csr_plan, F, x.device)
        L.call("regnn_spmm_fwd", L.ptr(rg.csr_ptr), L.ptr(rg.csr_idx), None, None, L.ptr(w_csr),
               None, None, None, L.ptr(x), L.ptr(y), rg.n_dst, F, L.dtype_code(x), *plan_args,
               L.stream())
        ctx.rg, ctx.ew_shape = rg, ew.shape
        ctx.save_for_backward(x, ewf)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, ewf = ctx.saved_tensors
        rg = ctx.rg
        gy = gy.contiguous().to(x.dtype)
        F = x.shape[1]
        gx = torch.empty(rg.n_src, F, dtype=x.dtype, device=x.device)
        w_csc = ewf[rg.csc_eid].contiguous()
        eg = torch.empty(rg.E, dtype=torch.float32, device=x.device) if ctx.needs_input_grad[1] else None
        plan_args, part = _plan_args(rg.csc_plan, F, x.device)
        L.call("regnn_spmm_bwd", L.ptr(rg.csc_ptr), L.ptr(rg.csc_idx), None, None, L.ptr(w_csc),
               None, None, L.ptr(gy), L.ptr(x), None, L.ptr(gx), None, 0, L.ptr(eg), None,
               rg.n_src, F, L.dtype_code(x), *plan_args, L.stream())
        g_ew = None
        if eg is not None:
            g_ew = torch.empty_like(eg)
            g_ew[rg.csc_eid] = eg
            g_ew = g_ew.view(ctx.ew_shape)
        return gx, g_ew, None


def edge_spmm(rg, x, ew):
    return _EdgeSpmm.apply(x, ew, rg)


# ---------------------------------------------------------------------------------------------
class _GatAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, el, er, ee_tab, rg, pack, slope, global_max=False):
        el, er = el.contiguous().float(), er.contiguous().float()
        H = el.shape[1]
        a = torch.empty(rg.E, H, dtype=torch.float32, device=el.device)
        t = None if ee_tab is None else ee_tab.detach().float().contiguous()
        rel = L.ptr(pack.rel_csr if t is not None else None)
        if global_max:
            # mag/utils.py:45-57: ONE max over every edge and head, + 1e-16 in the denominator
            s = torch.empty(rg.E, H, dtype=torch.float32, device=el.device)
            L.call("regnn_gat_scores", L.ptr(rg.csr_ptr), L.ptr(rg.csr_idx), rel, L.ptr(t),
                   L.ptr(el), L.ptr(er), rg.n_dst, H, float(slope), L.ptr(s), L.stream())
            gmax = s.amax().reshape(1) if s.numel() else torch.zeros(1, device=el.device)
            gp = _GatPlan(getattr(rg, "csr_plan", None), 2 * H, el.device)
            L.call("regnn_edge_softmax_fwd", L.ptr(rg.csr_ptr), L.ptr(s), None, None,
                   L.ptr(gmax), 1e-16, rg.n_dst, H, L.ptr(a), gp.ptr, L.stream())
        else:
            gp = _GatPlan(getattr(rg, "csr_plan", None), 2 * H, el.device)
            with timed("gat_softmax_fwd", rg.E * (5 + 12 * H) + rg.n_dst * 8 * H):
                L.call("regnn_gat_softmax_fwd", L.ptr(rg.csr_ptr), L.ptr(rg.csr_idx), rel,
                       L.ptr(t), L.ptr(el), L.ptr(er), rg.n_dst, H, float(slope), L.ptr(a),
                       gp.ptr, L.stream())
        ctx.rg, ctx.pack, ctx.slope = rg, pack, slope
        ctx.tab_shape = None if ee_tab is None else ee_tab.shape
        ctx.save_for_backward(el, er, t, a)
        return a

    @staticmethod
    def backward(ctx, ga):
        el, er, t, a = ctx.saved_tensors
        rg, H = ctx.rg, el.shape[1]
        ga = ga.contiguous().float()
        gs = torch.empty_like(a)
        ger = torch.empty_like(er)
        n_rel = t.shape[0] if t is not None else 0
        slab = _slab(n_rel * H, el.device) if (t is not None and ctx.needs_input_grad[2]) else None
        gp = _GatPlan(getattr(rg, "csr_plan", None), H, el.device)
        with timed("gat_softmax_bwd", rg.E * (5 + 16 * H) + rg.n_dst * 12 * H):
            L.call("regnn_gat_softmax_bwd", L.ptr(rg.csr_ptr), L.ptr(rg.csr_idx),
                   L.ptr(ctx.pack.rel_csr if t is not None else None), L.ptr(t), L.ptr(el),
                   L.ptr(er), L.ptr(a), L.ptr(ga), rg.n_dst, H, float(ctx.slope), L.ptr(gs),
                   L.ptr(ger), L.ptr(slab), n_rel, gp.ptr, L.stream())
        gel = torch.empty(rg.n_src, H, dtype=torch.float32, device=el.device)
        gq = _GatPlan(getattr(rg, "csc_plan", None), H, el.device)
        L.call("regnn_segment_sum", L.ptr(rg.csc_ptr), L.ptr(rg.csc2csr), L.ptr(gs), rg.n_src, H,
               L.ptr(gel), gq.ptr, L.stream())
        g_tab = _reduce(slab, n_rel * H).view(ctx.tab_shape) if slab is not None else None
        return gel, ger, g_tab, None, None, None, None


def gat_attention(rg, el, er, ee_tab=None, pack=None, slope=0.2, global_max=False):
    """a[e,h] (CSR edge order) = edge_softmax(leaky_relu(el[u]+er[v]+ee[rel_e], slope)).

    global_max: the ogbn-mag softmax (mag/utils.py:45-57, one max over all edges and heads,
    + 1e-16 in the denominator). Its backward is the per-destination formula: the global max's
    own gradient is 0 up to the 1e-16 term."""
    return _GatAttention.apply(el, er, ee_tab, rg, pack, slope, global_max)


# ---------------------------------------------------------------------------------------------
class _GatV2Score(torch.autograd.Function):
    """s[e,h] (CSR order) = <att[h], LeakyReLU(fs[u,h] + fd[v,h], slope)>."""

    @staticmethod
    def forward(ctx, fs, fd, att, rg, slope):
        N, H, D = fs.shape
        fs, fd = fs.contiguous().float(), fd.contiguous().float()
        a = att.detach().reshape(H * D).contiguous().float()
        s = torch.empty(rg.E, H, dtype=torch.float32, device=fs.device)
        gp = _GatPlan(getattr(rg, "csr_plan", None), 0, fs.device)     # hub rows as chunks
        with timed("gatv2_score_fwd", rg.E * (H * D * 4 + 4 * H + 4) + rg.n_dst * H * D * 4):
            L.call("regnn_gatv2_score_fwd", L.ptr(rg.csr_ptr), L.ptr(rg.csr_idx), L.ptr(fs),
                   L.ptr(fd), L.ptr(a), rg.n_dst, H, D, float(slope), L.ptr(s), gp.ptr,
                   L.stream())
        ctx.rg, ctx.slope, ctx.att_shape = rg, slope, att.shape
        ctx.save_for_backward(fs, fd, a)
        return s

    @staticmethod
    def backward(ctx, gs):
        fs, fd, a = ctx.saved_tensors
        rg, slope = ctx.rg, ctx.slope
        N, H, D = fs.shape
        gs = gs.contiguous().float()
        gfd = torch.empty_like(fd)
        gfs = torch.empty_like(fs)
        gp = _GatPlan(getattr(rg, "csr_plan", None), H * D, fs.device)
        gq = _GatPlan(getattr(rg, "csc_plan", None), H * D, fs.device)
        # with hub chunks the per-segment and the chunk pass take half the slab rows each
        rows = L.slab_rows() // (1 if gp.ptr is not None else 2)
        slab = torch.zeros(rows, H * D, dtype=torch.float32, device=fs.device)
        with timed("gatv2_score_bwd", 2 * rg.E * (H * D * 4 + 4 * H + 8) + 3 * rg.n_dst * H * D * 4):
            L.call("regnn_gatv2_score_bwd_dst", L.ptr(rg.csr_ptr), L.ptr(rg.csr_idx), L.ptr(fs),
                   L.ptr(fd), L.ptr(a), L.ptr(gs), rg.n_dst, H, D, float(slope), L.ptr(gfd),
                   L.ptr(slab), rows, gp.ptr, L.stream())
            L.call("regnn_gatv2_score_bwd_src", L.ptr(rg.csc_ptr), L.ptr(rg.csc_idx),
                   L.ptr(rg.csc2csr), L.ptr(fs), L.ptr(fd), L.ptr(a), L.ptr(gs), rg.n_src, H, D,
                   float(slope), L.ptr(gfs), gq.ptr, L.stream())
        g_att = _reduce(slab, H * D).view(ctx.att_shape)
        return gfs, gfd, g_att, None, None


def gatv2_scores(rg, fs, fd, att, slope=0.2):
    """GATv2 attention logits per edge (CSR order): layer/REGATv2Conv.py:139-141."""
    return _GatV2Score.apply(fs, fd, att, rg, slope)


class _EdgeSoftmax(torch.autograd.Function):
    """a = softmax over each destination's in-edges of z = s + ee[rel] (CSR order); per-segment
    max (DGL) or one global max + 1e-16 (ogbn-mag, mag/utils.py:45-57)."""

    @staticmethod
    def forward(ctx, s, ee_tab, rg, pack, global_max):
        s = s.contiguous().float()
        H = s.shape[1]
        t = None if ee_tab is None else ee_tab.detach().float().contiguous()
        rel = pack.rel_csr if t is not None else None
        a = torch.empty_like(s)
        gmax = None
        if global_max:
            z = s if t is None else s + t[rel.long()]
            gmax = z.amax().reshape(1) if z.numel() else torch.zeros(1, device=s.device)
        gp = _GatPlan(getattr(rg, "csr_plan", None), 2 * H, s.device)
        with timed("edge_softmax_fwd", rg.E * (8 * H + 1) + rg.n_dst * 8):
            L.call("regnn_edge_softmax_fwd", L.ptr(rg.csr_ptr), L.ptr(s), L.ptr(rel), L.ptr(t),
                   L.ptr(gmax), 1e-16 if global_max else 0.0, rg.n_dst, H, L.ptr(a), gp.ptr,
                   L.stream())
        ctx.rg, ctx.pack = rg, pack
        ctx.tab_shape = None if ee_tab is None else ee_tab.shape
        ctx.save_for_backward(a)
        return a

    @staticmethod
    def backward(ctx, ga):
        (a,) = ctx.saved_tensors
        rg, H = ctx.rg, a.shape[1]
        gz = torch.empty_like(a)
        need_tab = ctx.tab_shape is not None and ctx.needs_input_grad[1]
        n_rel = ctx.tab_shape[0] if need_tab else 0
        slab = _slab(n_rel * H, a.device) if need_tab else None
        gp = _GatPlan(getattr(rg, "csr_plan", None), H, a.device)
        with timed("edge_softmax_bwd", rg.E * (12 * H + 1) + rg.n_dst * 8):
            L.call("regnn_edge_softmax_bwd", L.ptr(rg.csr_ptr),
                   L.ptr(ctx.pack.rel_csr if need_tab else None), L.ptr(a),
                   L.ptr(ga.contiguous().float()), rg.n_dst, H, L.ptr(gz), L.ptr(slab), n_rel,
                   gp.ptr, L.stream())
        g_tab = _reduce(slab, n_rel * H).view(ctx.tab_shape) if need_tab else None
        return gz, g_tab, None, None, None


def edge_softmax_logits(rg, s, ee_tab=None, pack=None, global_max=False):
    """edge softmax of per-edge logits s [E, H] (CSR order) plus the relation bias ee[rel]."""
    return _EdgeSoftmax.apply(s, ee_tab, rg, pack, global_max)


class _AttnDots(torch.autograd.Function):
    """(el, er) = ((ft * attn_l).sum(-1), (ft * attn_r).sum(-1))  — layer/REGATConv.py:68-69."""

    @staticmethod
    def forward(ctx, ft, attn_l, attn_r):
        N, H, D = ft.shape
        ft = ft.contiguous().float()
        al = attn_l.detach().reshape(H, D).contiguous().float()
        ar = attn_r.detach().reshape(H, D).contiguous().float()
        el = torch.empty(N, H, dtype=torch.float32, device=ft.device)
        er = torch.empty_like(el)
        with timed("attn_dots_fwd", 4 * (N * H * D + 2 * N * H)):
            L.call("regnn_attn_dots_fwd", L.ptr(ft), L.ptr(al), L.ptr(ar), N, H, D, L.ptr(el),
                   L.ptr(er), L.stream())
        ctx.save_for_backward(ft, al, ar)
        ctx.shape = attn_l.shape
        return el, er

    @staticmethod
    def backward(ctx, gel, ger):
        ft, al, ar = ctx.saved_tensors
        N, H, D = ft.shape
        gel = torch.zeros(N, H, device=ft.device) if gel is None else gel.contiguous().float()
        ger = torch.zeros(N, H, device=ft.device) if ger is None else ger.contiguous().float()
        gft = torch.empty_like(ft)
        # one slab row per block: ~256+ rows per block, up to 2048 blocks (8 per CU)
        rows = max(1, min(2048, -(-N // 256)))
        slab = torch.empty(rows, 2 * H * D, dtype=torch.float32, device=ft.device)
        with timed("attn_dots_bwd", 4 * (2 * N * H * D + 2 * N * H)):
            L.call("regnn_attn_dots_bwd", L.ptr(ft), L.ptr(al), L.ptr(ar), L.ptr(gel), L.ptr(ger),
                   N, H, D, L.ptr(gft), L.ptr(slab), rows, L.stream())
        g = _reduce(slab, 2 * H * D)
        F = H * D
        return gft, g[:F].view(ctx.shape), g[F:].view(ctx.shape)


def attn_dots(ft, attn_l, attn_r):
    """el, er [N, H] of the GAT attention (ft [N, H, D], attn_* [1, H, D])."""
    return _AttnDots.apply(ft, attn_l, attn_r)


class _HeadSpmm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, ft, rg):
        N, H, D = ft.shape
        ft = ft.contiguous()
        a = a.contiguous().float()
        y = torch.empty(rg.n_dst, H, D, dtype=ft.dtype, device=ft.device)
        s_ = ft.element_size()
        with timed("spmm_heads_fwd", rg.E * (H * D * s_ + 4 * H + 4) + rg.n_dst * (H * D * s_ + 4)):
            gp = _GatPlan(getattr(rg, "csr_plan", None), H * D, ft.device)
            L.call("regnn_spmm_heads_fwd", L.ptr(rg.csr_ptr), L.ptr(rg.csr_idx), None, L.ptr(a),
                   L.ptr(ft), L.ptr(y), rg.n_dst, H, D, L.dtype_code(ft), gp.ptr, L.stream())
        ctx.rg = rg
        ctx.save_for_backward(a, ft)
        return y

    @staticmethod
    def backward(ctx, gy):
        a, ft = ctx.saved_tensors
        rg = ctx.rg
        N, H, D = ft.shape
        gy = gy.contiguous().to(ft.dtype)
        gft = torch.empty_like(ft)
        ga = torch.empty_like(a)
        s_ = ft.element_size()
        with timed("spmm_heads_bwd",
                   rg.E * (H * D * s_ + 8 * H + 8) + rg.n_src * (2 * H * D * s_ + 4)):
            gq = _GatPlan(getattr(rg, "csc_plan", None), H * D, ft.device)
            L.call("regnn_spmm_heads_bwd", L.ptr(rg.csc_ptr), L.ptr(rg.csc_idx),
                   L.ptr(rg.csc2csr), L.ptr(a), L.ptr(gy), L.ptr(ft), L.ptr(gft), L.ptr(ga),
                   rg.n_src, H, D, L.dtype_code(ft), gq.ptr, L.stream())
        return ga, gft, None


class _GatFused(torch.autograd.Function):
    """out[v,h,:] = sum_{e: u->v} edge_softmax(LeakyReLU(el[u]+er[v]+ee[rel]))[e,h] * ft[u,h,:]
    in one pass (regnn_gat_fused_fwd, online softmax; the [E, H] attention is not stored). The
    backward re-forms the attention from the per-(destination, head) log-sum-exp
    (regnn_gat_attn_lse) and runs the unfused backward kernels."""

    @staticmethod
    def forward(ctx, el, er, ee_tab, ft, rg, pack, slope, attn_l):
        N, H, D = ft.shape
        el, er, ft = el.contiguous().float(), er.contiguous().float(), ft.contiguous()
        al = None if attn_l is None else attn_l.detach().reshape(H, D).float().contiguous()
        t = None if ee_tab is None else ee_tab.detach().float().contiguous()
        rel = pack.rel_csr if t is not None else None
        out = torch.empty(rg.n_dst, H, D, dtype=ft.dtype, device=ft.device)
        lse = torch.empty(rg.n_dst, H, dtype=torch.float32, device=ft.device)
        s_ = ft.element_size()
        with timed("gat_fused_fwd", rg.E * (H * D * s_ + 4 * H + 5) +
                   rg.n_dst * (H * D * s_ + 8 * H + 4)):
            gp = _GatPlan(getattr(rg, "csr_plan", None), H * D + 2 * H, ft.device)
            L.call("regnn_gat_fused_fwd", L.ptr(rg.csr_ptr), L.ptr(rg.csr_idx), L.ptr(rel),
                   L.ptr(t), L.ptr(el), L.ptr(er), L.ptr(ft), L.ptr(out), L.ptr(lse), rg.n_dst, H,
                   D, float(slope), L.dtype_code(ft), L.ptr(al), gp.ptr, L.stream())
        ctx.rg, ctx.pack, ctx.slope = rg, pack, slope
        ctx.tab_shape = None if ee_tab is None else ee_tab.shape
        ctx.save_for_backward(el, er, t, ft, lse)
        return out

    @staticmethod
    def backward(ctx, gy):
        el, er, t, ft, lse = ctx.saved_tensors
        rg, pack, slope = ctx.rg, ctx.pack, ctx.slope
        N, H, D = ft.shape
        rel = pack.rel_csr if t is not None else None
        a = torch.empty(rg.E, H, dtype=torch.float32, device=ft.device)
        with timed("gat_attn_lse", rg.E * (5 + 8 * H) + rg.n_dst * 8 * H):
            gp0 = _GatPlan(getattr(rg, "csr_plan", None), 0, ft.device)   # alive for the call
            L.call("regnn_gat_attn_lse", L.ptr(rg.csr_ptr), L.ptr(rg.csr_idx), L.ptr(rel),
                   L.ptr(t), L.ptr(el), L.ptr(er), L.ptr(lse), rg.n_dst, H, float(slope),
                   L.ptr(a), gp0.ptr, L.stream())
        gy = gy.contiguous().to(ft.dtype)
        gft = torch.empty_like(ft)
        ga = torch.empty_like(a)
        s_ = ft.element_size()
        with timed("spmm_heads_bwd",
                   rg.E * (H * D * s_ + 8 * H + 8) + rg.n_src * (2 * H * D * s_ + 4)):
            gq = _GatPlan(getattr(rg, "csc_plan", None), H * D, ft.device)
            L.call("regnn_spmm_heads_bwd", L.ptr(rg.csc_ptr), L.ptr(rg.csc_idx),
                   L.ptr(rg.csc2csr), L.ptr(a), L.ptr(gy), L.ptr(ft), L.ptr(gft), L.ptr(ga),
                   rg.n_src, H, D, L.dtype_code(ft), gq.ptr, L.stream())
        gs = torch.empty_like(a)
        ger = torch.empty_like(er)
        n_rel = t.shape[0] if t is not None else 0
        slab = _slab(n_rel * H, el.device) if (t is not None and ctx.needs_input_grad[2]) else None
        with timed("gat_softmax_bwd", rg.E * (5 + 16 * H) + rg.n_dst * 12 * H):
            gp = _GatPlan(getattr(rg, "csr_plan", None), H, el.device)
            L.call("regnn_gat_softmax_bwd", L.ptr(rg.csr_ptr), L.ptr(rg.csr_idx), L.ptr(rel),
                   L.ptr(t), L.ptr(el), L.ptr(er), L.ptr(a), L.ptr(ga), rg.n_dst, H,
                   float(slope), L.ptr(gs), L.ptr(ger), L.ptr(slab), n_rel, gp.ptr, L.stream())
        gel = torch.empty(rg.n_src, H, dtype=torch.float32, device=el.device)
        gq = _GatPlan(getattr(rg, "csc_plan", None), H, el.device)
        L.call("regnn_segment_sum", L.ptr(rg.csc_ptr), L.ptr(rg.csc2csr), L.ptr(gs), rg.n_src, H,
               L.ptr(gel), gq.ptr, L.stream())
        g_tab = _reduce(slab, n_rel * H).view(ctx.tab_shape) if slab is not None else None
        return gel, ger, g_tab, gft, None, None, None, None


def gat_fused(rg, el, er, ft, ee_tab=None, pack=None, slope=0.2, attn_l=None):
    """layer/REGATConv.py:80-92 without attention dropout, as one fused forward pass (H a power of
    two <= 32; otherwise the unfused gat_attention + head_spmm). With attn_l (el then being
    attn_dots(ft, attn_l, ...)'s) the kernel re-forms el from the rows it gathers, bitwise the
    same, instead of reading it per edge (fp32 rows, D / 4 a power of two)."""
    H = ft.shape[1]
    if H & (H - 1) or H > 32:
        return head_spmm(rg, gat_attention(rg, el, er, ee_tab, pack, slope), ft)
    return _GatFused.apply(el, er, ee_tab, ft, rg, pack, slope, attn_l)


def head_spmm(rg, a, ft):
    """out[v,h,:] = sum_{e: u->v} a[e,h] * ft[u,h,:]   (a in CSR edge order)."""
    return _HeadSpmm.apply(a, ft, rg)


# ---------------------------------------------------------------------------------------------
def col_sum(x):
    """x.sum(0) for a tall row-major fp32 matrix, deterministic (HIP col_sum + slab reduce)."""
    x = x.contiguous().float()
    rows, cols = x.shape
    slab = torch.zeros(L.slab_rows() // 2, cols, dtype=torch.float32, device=x.device)
    L.call("regnn_col_sum", L.ptr(x), rows, cols, L.ptr(slab), L.stream())
    return _reduce(slab, cols)


def linear_wgrad(g, x):
    """(g^T x, g.sum(0)) of a Linear's backward over tall row-major g [n, C], x [n, K]:
    regnn_linear_wgrad (one fp32-accurate MFMA pass, fixed-order slab reduce) for C <= 64 and
    K in {64, 128, 256}, else a chunked GEMM + col_sum. fp32 results."""
    n, C = g.shape
    K = x.shape[1]
    aligned = g.dtype == torch.float32 or (g.stride(0) % 4 == 0 and g.data_ptr() % 8 == 0)
    if (g.is_cuda and C <= 64 and K in (64, 128, 256) and g.dtype == x.dtype
            and g.dtype in (torch.float32, torch.bfloat16) and g.stride(1) == 1 and aligned):
        x = x.contiguous()
        width = 64 * K + 64
        rows = L.slab_rows() // 2
        slab = torch.zeros(rows, width, dtype=torch.float32, device=g.device)
        with timed("linear_wgrad", (n * (C + K)) * g.element_size()):
            L.call("regnn_linear_wgrad", L.ptr(g), n, C, g.stride(0), L.ptr(x), K,
                   L.dtype_code(g), L.ptr(slab), rows, L.stream())
            tot = _reduce(slab, width)
        return tot[:64 * K].view(64, K)[:C], tot[64 * K:64 * K + C]
    return batched_wgrad(g.float(), x.float()), col_sum(g)


# ---------------------------------------------------------------------------------------------
class _HeadCE(torch.autograd.Function):
    """(logits, loss) = (h W^T + b over ALL rows, mean CE over the first n rows vs labels).

    The training step of run_regnn.py (:146-150) computes out_lin on every node and the loss on the
    train rows; autograd through that slice materialises an all-rows zero-filled logits gradient
    (19.4M x 349 fp32 = 27 GB at mag-10x) and runs the backward GEMMs over it. This op returns the
    same logits and loss and the same gradients: one HIP pass (regnn_softmax_xent) forms the loss
    rows and the scaled softmax gradient of the loss rows only. The logits output is
    non-differentiable: use it for evaluation, the loss for training."""

    @staticmethod
    def forward(ctx, h, W, b, labels):
        ctx.set_materialize_grads(False)          # no all-rows zero gradient for `logits`
        n, C = labels.numel(), W.shape[0]
        dev = h.device
        loss_rows = torch.empty(n, dtype=torch.float32, device=dev)
        lab = labels.to(torch.int64).contiguous()
        hin = h
        ctx.in_dtype = h.dtype
        if head_fused(h.shape[1], C) and (h.dtype == torch.float32 or (
                h.dtype == torch.bfloat16 and HEAD["p"] == "z")):
            # bf16 rows (a bf16 feature pipeline, z mode only) are read as they are and get a
            # bf16 gradient back (regnn_head_fwd_lse / regnn_head_bwd_z dtype)
            h = h.contiguous()
            Wc = W.detach().contiguous()
            # rows padded to 16 classes (64-byte aligned): logits is a [rows, C] view of it
            ld = 16 * ((C + 15) // 16)
            logits = torch.empty(h.shape[0], ld, dtype=torch.float32, device=dev)[:, :C]
            bp = L.ptr(b.detach().contiguous()) if b is not None else None
            if HEAD["p"] == "z":
                # no p rows: the backward re-forms them from these logits rows and the lse
                buf = torch.empty(2, n, dtype=torch.float32, device=dev)
                loss_rows = buf[0]
                p = None
                with timed("head_fwd", h.numel() * h.element_size() +
                           4 * (h.shape[0] * C + 2 * n) + 8 * n):
                    L.call("regnn_head_fwd_lse", L.ptr(h), h.shape[0], h.shape[1], L.ptr(Wc),
                           bp, C, ld, L.ptr(lab), n, L.ptr(logits), L.ptr(buf),
                           L.dtype_code(h), L.stream())
                ctx.zsrc = (logits, logits._version, buf[1], lab)
            else:
                p = torch.empty(n, ld, dtype=torch.float32, device=dev)[:, :C]
                nbytes = 4 * (h.numel() + h.shape[0] * C + n * C + n) + 8 * n
                with timed("head_fwd", nbytes):
                    L.call("regnn_head_fwd", L.ptr(h), h.shape[0], h.shape[1], L.ptr(Wc), bp,
                           C, ld, L.ptr(lab), n, 1.0 / n, L.ptr(logits), L.ptr(p),
                           L.ptr(loss_rows), L.stream())
        else:
            p = torch.empty(n, C, dtype=torch.float32, device=dev)
            logits = torch.addmm(b, h, W.t()) if b is not None else h @ W.t()
            with timed("softmax_xent", n * C * 8):
                L.call("regnn_softmax_xent", L.ptr(logits), n, C, logits.stride(0), L.ptr(lab),
                       1.0 / n, L.ptr(p), L.ptr(loss_rows), L.stream())
        loss = loss_rows.sum() / n
        ctx.save_for_backward(h, W, p)
        ctx.n, ctx.C = n, C
        ctx.bias = b.detach() if b is not None else None
        ctx.has_bias = b is not None
        # h straight from an aggregation (re_spmm): its backward row pass rides on gh's kernel
        ctx.link = getattr(hin, "_regnn_link", None) if (
            hin.dtype == torch.float32 or getattr(ctx, "zsrc", None) is not None) else None
        ctx.hx = None
        ctx.mark_non_differentiable(logits)
        return logits, loss

    @staticmethod
    def backward(ctx, _g_logits, g_loss):
        h, W, p = ctx.saved_tensors
        n, C = ctx.n, ctx.C
        K = h.shape[1]
        gh = gW = gb = None
        if g_loss is None:
            return None, None, None, None
        need_h, need_w = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        need_b = ctx.has_bias and ctx.needs_input_grad[2]
        zsrc = getattr(ctx, "zsrc", None)
        if zsrc is not None:
            # kept until the graph is freed: a retain_graph backward re-forms p from z again
            z, ver, lse, lab = zsrc
            if z._version == ver:
                return _head_bwd_z(ctx, h, W, z, lse, lab, g_loss, need_h, need_w, need_b)
            # the caller modified the logits in place: re-form p from h (the stored-p path)
            if ctx.in_dtype != torch.float32:
                ctx.link = None                    # the fp32 hand-off kernels do not apply
                h = h.float()
            zf = torch.addmm(ctx.bias, h[:n], W.detach().t()) if ctx.bias is not None else \
                h[:n] @ W.detach().t()
            p = torch.empty(n, C, dtype=torch.float32, device=h.device)
            lr = torch.empty(n, dtype=torch.float32, device=h.device)
            L.call("regnn_softmax_xent", L.ptr(zf), n, C, zf.stride(0), L.ptr(lab), 1.0 / n,
                   L.ptr(p), L.ptr(lr), L.stream())
        if head_fused(K, C) and h.dtype == torch.float32:
            # regnn_head_bwd: gh = g_loss * p W (rows >= n zero-filled in the same launch) and
            # the (p^T h | colsum p) slab, each kernel reading p once (fp32 MFMA)
            Cp = 16 * ((C + 15) // 16)
            rows = 2048
            slab = (torch.zeros(rows, Cp * K + Cp, dtype=torch.float32, device=p.device)
                    if (need_w or need_b) else None)
            hc = h.contiguous()
            if need_h:
                gh = torch.empty_like(h)
                gl = g_loss.detach().reshape(1).float().contiguous()
                nx = ctx.link
                if nx is not None and nx.post.numel() == h.shape[0] and \
                        PRESCALE["next"] != "off":
                    # also nx.post * gh and <gh, h> / nx.post for h's producer (_NextLink)
                    nx_out = torch.empty_like(h)
                    nx_dot = torch.empty(h.shape[0], dtype=torch.float32, device=h.device)
                    with timed("head_gh", 4 * (p.numel() + h.numel())):
                        L.call("regnn_head_gh_next", L.ptr(p), n, C, p.stride(0), K,
                               L.ptr(W.detach().contiguous()), L.ptr(gl), L.ptr(gh),
                               h.shape[0], L.ptr(nx.post), L.ptr(hc), L.ptr(nx_out),
                               L.ptr(nx_dot), L.stream())
                    nx.handoff = (gh, gh._version, nx_out, nx_dot, n)
                else:
                    with timed("head_gh", 4 * (p.numel() + h.numel())):
                        L.call("regnn_head_bwd", L.ptr(p), n, C, p.stride(0), K,
                               L.ptr(W.detach().contiguous()), None, L.ptr(gl), L.ptr(gh),
                               h.shape[0], None, 0, L.stream())
            if slab is not None:
                with timed("head_bwd", 4 * (p.numel() + n * K)):
                    L.call("regnn_head_bwd", L.ptr(p), n, C, p.stride(0), K, None, L.ptr(hc),
                           None, None, 0, L.ptr(slab), rows, L.stream())
            if slab is not None:
                tot = _reduce(slab, Cp * K + Cp)
                if need_w:
                    gW = tot[:Cp * K].view(Cp, K)[:C] * g_loss
                if need_b:
                    gb = tot[Cp * K:Cp * K + C] * g_loss
            if gh is not None and gh.dtype != ctx.in_dtype:
                gh = gh.to(ctx.in_dtype)
            return gh, gW, gb, None
        if need_h:
            gh = torch.empty_like(h)
            gh[n:].zero_()
            torch.mm(p, W * g_loss, out=gh[:n])      # g_loss folded into the C x K weight
            if gh.dtype != ctx.in_dtype:
                gh = gh.to(ctx.in_dtype)
        if need_w:
            gW = batched_wgrad(p, h[:n]) * g_loss
        if need_b:
            gb = col_sum(p) * g_loss
        return gh, gW, gb, None


# "z": regnn_head_fwd_lse stores no p rows, the backward kernels re-form p from the logits rows
# (regnn_head_bwd_z); "p": p stored by the forward and read back (regnn_head_fwd / _bwd)
HEAD = {"p": os.environ.get("REGNN_HEAD_P", "z")}


def _head_bwd_z(ctx, h, W, z, lse, lab, g_loss, need_h, need_w, need_b):
    """_HeadCE.backward from the logits rows z [n, C] (stride ld) and their lse."""
    n, C = ctx.n, ctx.C
    K = h.shape[1]
    gh = gW = gb = None
    Cp = 16 * ((C + 15) // 16)
    rows = 2048
    hc = h.contiguous()
    hx = ctx.hx if ctx.hx is not None else hc        # rows in the caller's storage dtype
    zp, ld = L.ptr(z), z.stride(0)
    if need_h:
        gh = torch.empty_like(hx)
        gl = g_loss.detach().reshape(1).float().contiguous()
        nx = ctx.link
        nx_args = (None, None, None)
        if nx is not None and nx.post.numel() == h.shape[0] and PRESCALE["next"] != "off":
            nx_out = torch.empty_like(hx)
            nx_dot = torch.empty(h.shape[0], dtype=torch.float32, device=h.device)
            nx_args = (L.ptr(nx.post), L.ptr(nx_out), L.ptr(nx_dot))
        with timed("head_gh", 4 * n * C + (2 if nx_args[0] is not None else 1) * gh.numel() *
                   gh.element_size()):
            L.call("regnn_head_bwd_z", zp, n, C, ld, K, L.ptr(W.detach().contiguous()),
                   L.ptr(hc), L.ptr(gl), L.ptr(gh), h.shape[0], None, 0, L.ptr(lse),
                   L.ptr(lab), 1.0 / n, L.ptr(hx), *nx_args, L.dtype_code(hx), L.stream())
        if nx_args[0] is not None:
            nx.handoff = (gh, gh._version, nx_out, nx_dot, n)
    if need_w or need_b:
        slab = torch.zeros(rows, Cp * K + Cp, dtype=torch.float32, device=h.device)
        with timed("head_bwd", 4 * (n * C + n * K)):
            L.call("regnn_head_bwd_z", zp, n, C, ld, K, None, L.ptr(hc), None, None, 0,
                   L.ptr(slab), rows, L.ptr(lse), L.ptr(lab), 1.0 / n, None, None, None, None,
                   L.dtype_code(hc), L.stream())
        tot = _reduce(slab, Cp * K + Cp)
        if need_w:
            gW = tot[:Cp * K].view(Cp, K)[:C] * g_loss
        if need_b:
            gb = tot[Cp * K:Cp * K + C] * g_loss
    return gh, gW, gb, None


def head_argmax(h, weight, bias=None):
    """argmax_c (h W^T + b) per row without the logits tensor (regnn_head_argmax), int64."""
    h = h.detach().contiguous().float()
    out = torch.empty(h.shape[0], dtype=torch.int64, device=h.device)
    C = weight.shape[0]
    if not head_fused(h.shape[1], C):
        return torch.addmm(bias, h, weight.t()).argmax(-1) if bias is not None else \
            (h @ weight.t()).argmax(-1)
    with timed("head_argmax", 4 * (h.numel() + C * h.shape[1]) + 8 * h.shape[0]):
        L.call("regnn_head_argmax", L.ptr(h), h.shape[0], h.shape[1],
               L.ptr(weight.detach().float().contiguous()),
               L.ptr(None if bias is None else bias.detach().float().contiguous()), C,
               L.ptr(out), L.stream())
    return out


def head_fused(K, C):
    """shapes regnn_head_fwd takes (include/regnn_hip.h): K = 64, C <= 384."""
    return K == 64 and 0 < C <= 384


def batched_wgrad(g, x, chunk=1 << 15):
    """g^T x for tall g [rows, m], x [rows, k]: a batched GEMM over row chunks + a fixed-order
    sum (one (m, k) GEMM with K = rows ~ 1e7 ran at ~1 TB/s in hipBLASLt, profiled)."""
    rows = g.shape[0]
    nb = rows // chunk
    if nb < 2:
        return g.t() @ x
    main = nb * chunk
    part = torch.bmm(g[:main].view(nb, chunk, -1).transpose(1, 2), x[:main].view(nb, chunk, -1))
    out = part.sum(0)
    if main < rows:
        out = out + g[main:].t() @ x[main:]
    return out


def head_ce(h, weight, bias, labels, rows=None):
    """fused output head + cross-entropy -> (logits of every row, mean loss over the loss rows).

    rows = None: the loss rows are [0, len(labels)) (run_regnn.py:146-148 with the train nodes
    numbered first, e.g. by data.loss_rows_first): the fast path, whose backward hands the last
    aggregation its gradient rows and gathers only the CSC edges into the loss rows.
    rows = an index tensor (any train split): the loss rows h[rows] go through the same fused
    head (labels[i] is the label of row rows[i]); the logits of every row are returned without
    a gradient, and the gradient reaches h through the gather (no hand-off).
    bf16 rows go in as they are (z mode: widened inside, bf16 gradient out), else as fp32."""
    if h.dtype != torch.float32 and not (h.dtype == torch.bfloat16 and HEAD["p"] == "z" and
                                         head_fused(h.shape[-1], weight.shape[0])):
        h = h.float()
    if rows is not None:
        rows = rows.to(h.device, torch.int64).reshape(-1)
        n = rows.numel()
        if n != labels.numel():
            raise ValueError(f"{n} loss rows but {labels.numel()} labels")
        if not (n <= h.shape[0] and bool((rows == torch.arange(n, device=rows.device)).all())):
            _, loss = _HeadCE.apply(h.index_select(0, rows), weight, bias, labels)
            with torch.no_grad():
                logits = h.float() @ weight.detach().t()
                if bias is not None:
                    logits += bias.detach()
            return logits, loss
    return _HeadCE.apply(h, weight, bias, labels)


# ---------------------------------------------------------------------------------------------
# per-node-type input rows of the ogbn-mag path (mag/regnn_ns.py:300-326, REGNN.group_input)
def _ptr_array(ptrs):
    return (ctypes.c_void_p * len(ptrs))(*[p if p else None for p in ptrs])


def _i32(t):
    return t if t.dtype == torch.int32 and t.is_contiguous() else t.to(torch.int32).contiguous()


def _i64(t):
    return t if t.dtype == torch.int64 and t.is_contiguous() else t.to(torch.int64).contiguous()


class _TypedGather(torch.autograd.Function):
    """out[i] = tables[type(i)][local(i)] (regnn_typed_gather; rows of types without a table
    are zero, as mag/regnn_ns.py:307's zeros); the backward adds the row gradients into the
    tables that learn (feats_type-2 embeddings, regnn_typed_scatter)."""

    @staticmethod
    def forward(ctx, n_id, node_type, local_idx, K, *tables):
        n = node_type.numel() if n_id is None else n_id.numel()
        out = torch.empty(n, K, dtype=torch.float32, device=node_type.device)
        L.call("regnn_typed_gather", L.ptr(n_id), n, L.ptr(node_type), L.ptr(local_idx),
               len(tables), _ptr_array([L.ptr(t) for t in tables]), K, L.ptr(out), L.stream())
        ctx.save_for_backward(n_id, node_type, local_idx)
        ctx.shapes = [None if t is None else t.shape for t in tables]
        ctx.K = K
        return out

    @staticmethod
    def backward(ctx, g):
        n_id, node_type, local_idx = ctx.saved_tensors
        need = ctx.needs_input_grad[4:]
        grads = [torch.zeros(s, dtype=torch.float32, device=g.device) if (s is not None and nd)
                 else None for s, nd in zip(ctx.shapes, need)]
        if any(x is not None for x in grads):
            g = g.contiguous().float()
            L.call("regnn_typed_scatter", L.ptr(n_id), g.shape[0], L.ptr(node_type),
                   L.ptr(local_idx), len(grads), _ptr_array([L.ptr(x) for x in grads]), ctx.K,
                   L.ptr(g), L.stream())
        return (None, None, None, None, *grads)


def typed_gather(tables, node_type, local_idx, n_id=None):
    """rows of the per-type tables for every node of n_id (all nodes when None): the feats_type-2
    input matrix of mag/regnn_ns.py:307-314 in one launch, no per-type masks or host syncs.
    tables: list indexed by node type (None: zero rows), fp32 [*, K] contiguous."""
    K = next(t.shape[1] for t in tables if t is not None)
    tabs = [None if t is None else t.contiguous() for t in tables]
    nid = None if n_id is None else _i64(n_id)
    return _TypedGather.apply(nid, _i64(node_type), _i64(local_idx), K, *tabs)


def typed_plan(node_type, local_idx, n_id, T):
    """rows sorted by node type (stable): (order, src, type_off) of regnn_typed_linear_*, built
    with device ops only (no host synchronisation)."""
    t = node_type if n_id is None else node_type[n_id]
    l = local_idx if n_id is None else local_idx[n_id]
    t = t.to(torch.int64)
    order = torch.argsort(t, stable=True)
    src = l.to(torch.int64)[order].contiguous()
    cnt = torch.zeros(T, dtype=torch.int64, device=t.device)
    cnt.scatter_add_(0, t, torch.ones_like(t))
    off = torch.zeros(T + 1, dtype=torch.int32, device=t.device)
    off[1:] = torch.cumsum(cnt, 0).to(torch.int32)
    return order.contiguous(), src, off, t.numel()


class _TypedLinear(torch.autograd.Function):
    """Y[i] = tables[t_i][local_i] W[g(t_i)]^T + b[g(t_i)]: group_input's per-type Linear
    (mag/regnn_ns.py:316-324) as one gather-fused fp32-MFMA launch over the type-sorted rows
    (regnn_typed_linear_fwd); the backward's weight / bias gradients per weight group by
    regnn_typed_linear_wgrad (fixed-order chunk partials)."""

    @staticmethod
    def forward(ctx, plan, tables, wg, G, *params):
        order, src, off, n = plan
        Ws, bs = params[:G], params[G:]
        O, K = Ws[0].shape
        dev = Ws[0].device
        Y = torch.empty(n, O, dtype=torch.float32, device=dev)
        T = len(tables)
        Wd = [W.detach().contiguous() for W in Ws]
        bd = [None if b is None else b.detach().contiguous() for b in bs]
        with timed("typed_linear", n * (K + O) * 4):
            L.call("regnn_typed_linear_fwd", L.ptr(order), L.ptr(src), L.ptr(off), n, T,
                   _ptr_array([L.ptr(t) for t in tables]),
                   _ptr_array([L.ptr(Wd[wg[t]]) for t in range(T)]),
                   _ptr_array([L.ptr(bd[wg[t]]) for t in range(T)]), K, O, L.ptr(Y), L.stream())
        ctx.plan, ctx.tables, ctx.wg, ctx.G = plan, tables, wg, G
        ctx.shape = (O, K)
        ctx.has_b = [b is not None for b in bs]
        return Y

    @staticmethod
    def backward(ctx, gY):
        order, src, off, n = ctx.plan
        G, (O, K) = ctx.G, ctx.shape
        T = len(ctx.tables)
        gY = gY.contiguous().float()
        dev = gY.device
        gW = [torch.empty(O, K, dtype=torch.float32, device=dev) for _ in range(G)]
        gb = [torch.empty(O, dtype=torch.float32, device=dev) if hb else None
              for hb in ctx.has_b]
        slab = torch.empty(L.typed_slab_floats(n, T, K, O), dtype=torch.float32, device=dev)
        with timed("typed_wgrad", n * (K + O) * 4):
            L.call("regnn_typed_linear_wgrad", L.ptr(order), L.ptr(src), L.ptr(off), n, T,
                   _ptr_array([L.ptr(t) for t in ctx.tables]), (ctypes.c_int32 * T)(*ctx.wg),
                   G, K, O, L.ptr(gY), L.ptr(slab), _ptr_array([L.ptr(x) for x in gW]),
                   _ptr_array([L.ptr(x) for x in gb]), L.stream())
        return (None, None, None, None, *gW, *gb)


def typed_linear_fusable(tables, weights, biases):
    """regnn_typed_linear's shapes: <= 8 types, every table fp32 contiguous [*, K] on the device
    with no gradient, K in {64, 128, 256}, weights [O, K] with O a multiple of 64."""
    if not 0 < len(tables) <= 8 or any(t is None for t in tables):
        return False
    K = tables[0].shape[1]
    O = weights[0].shape[0]
    return (K in (64, 128, 256) and O % 64 == 0
            and all(t.is_cuda and t.dtype == torch.float32 and t.dim() == 2 and t.shape[1] == K
                    and t.is_contiguous() and not t.requires_grad for t in tables)
            and all(W.shape == (O, K) and W.dtype == torch.float32 for W in weights)
            and all(b is None or (b.shape == (O,) and b.dtype == torch.float32) for b in biases))


def typed_linear(tables, weights, biases, node_type, local_idx, n_id=None, wgroup=None):
    """tables[t][local] @ weights[g(t)].T + biases[g(t)] for every node of n_id (wgroup: type ->
    weight index, default the identity): group_input's per-type Linear over the sampled nodes."""
    T = len(tables)
    wg = list(range(T)) if wgroup is None else [int(g) for g in wgroup]
    plan = typed_plan(node_type, local_idx, n_id, T)
    return _TypedLinear.apply(plan, [t.contiguous() for t in tables], wg, len(weights),
                              *weights, *biases)


# ---------------------------------------------------------------------------------------------
# fp32-accurate dense products on bf16 MFMA (regnn_gemm_x6, bf16x6): the wide NS model's GEMMs
# ---------------------------------------------------------------------------------------------
# "on": ops.mm runs regnn_gemm_x6 where it applies; "off": torch (hipBLASLt fp32), A/B
GEMM_X6 = {"mode": os.environ.get("REGNN_GEMM_X6", "on")}


# split-K target: blocks (tile x split) per launch; env REGNN_GEMM_SPLIT_TARGET for A/B runs
_SPLIT_TARGET = int(os.environ.get("REGNN_GEMM_SPLIT_TARGET", "512"))


# typical live rows of a capacity-sized operand: LIVE_HINT[M] = rows (set_live_hint; the NS
# trainer's module path sets it from its first batch when ns.GEMM_LIVE_HINT is on -- measured
# slower, off by default). The split-K factor of every GEMM with M rows is chosen for that many
# rows (the dead row tiles the kernel skips leave much of the chip idle: 13312-row capacity, ~6 k
# live rows at mag-10x), whether or not the call passes m_live, so a product's summation order
# depends on M alone; with split-K the dead row tiles write no partial and the reduce skips them
LIVE_HINT = {}


def set_live_hint(capacity_rows, rows):
    LIVE_HINT[int(capacity_rows)] = max(1, min(int(capacity_rows), int(rows)))


def _gemm_splits(M, N, K):
    """split-K factor: about two 128 x 128 tiles per CU for a small output over a long
    reduction (each split keeps >= 4 k-steps of 32); M at its live-row hint (LIVE_HINT)."""
    M = LIVE_HINT.get(M, M)
    tiles = -(-M // 128) * -(-N // 128)
    nk = -(-K // 32)
    if tiles >= 256 or nk < 8:
        return 1
    return int(max(1, min(64, _SPLIT_TARGET // tiles, nk // 4)))


def gemm_x6(a, b, trans_a=False, trans_b=False, out=None, beta=0.0, m_live=None, k_live=None):
    """op(a) @ op(b) (+ beta * out) in fp32 accuracy: a [M, K] ([K, M] with trans_a), b [K, N]
    ([N, K] with trans_b), contiguous fp32 device tensors. m_live / k_live: one-element int32
    device tensors, the live rows of op(a) / the live k (the operands are zero past them: a
    capacity-sized sampled block's unused rows), so the kernel skips those products."""
    M, K = (a.shape[1], a.shape[0]) if trans_a else (a.shape[0], a.shape[1])
    Kb, N = (b.shape[1], b.shape[0]) if trans_b else (b.shape[0], b.shape[1])
    if K != Kb:
        raise ValueError(f"gemm_x6: inner dimensions {K} and {Kb} differ")
    if out is None:
        out = torch.empty(M, N, dtype=torch.float32, device=a.device)
        beta = 0.0
    S = _gemm_splits(M, N, K)
    work = (torch.empty(int(L._so.regnn_gemm_x6_work_floats(M, N, S)), dtype=torch.float32,
                        device=a.device) if S > 1 else None)
    L.call("regnn_gemm_x6", int(trans_a), int(trans_b), M, N, K, L.ptr(a), a.stride(0), L.ptr(b),
           b.stride(0), L.ptr(out), out.stride(0), float(beta), L.ptr(work), S, L.ptr(m_live),
           L.ptr(k_live), L.stream())
    return out


# "on": ops.mm's live-row hint reaches the GEMMs (the capacity-sized block's unused rows are
# skipped); "off": every row computed (A/B)
LIVE_ROWS = {"mode": os.environ.get("REGNN_GEMM_LIVE_ROWS", "on")}


def gemm_x6_ok(*ts):
    """the operands regnn_gemm_x6 takes: 2-D contiguous fp32 device tensors (rows of a multiple
    of 4 floats on 16-byte boundaries load as vectors, any others per element)."""
    return all(t is not None and t.is_cuda and t.dtype == torch.float32 and t.dim() == 2 and
               t.is_contiguous() for t in ts)


class _MMx6(torch.autograd.Function):
    """c + a @ b (c optional, broadcast over rows when 1-D) with regnn_gemm_x6 forward and
    backward (ga = g b^T, gb = a^T g: split-K over the rows). live: a's live rows (a one-element
    int32 device tensor, or None): a's rows past it are zero, the output's rows there are c's
    (the incoming gradient's rows there are taken as zero: nothing reads them)."""

    @staticmethod
    def forward(ctx, a, b, c, live):
        if c is None:
            out = gemm_x6(a, b, m_live=live)
        else:
            out = (c.expand(a.shape[0], b.shape[1]) if c.dim() == 1 else c).contiguous().clone()
            gemm_x6(a, b, out=out, beta=1.0, m_live=live)
        ctx.save_for_backward(a, b)
        ctx.c_shape = None if c is None else c.shape
        ctx.live = live
        return out

    @staticmethod
    def backward(ctx, g):
        a, b = ctx.saved_tensors
        g = g.contiguous()
        live = ctx.live
        ga = gemm_x6(g, b, trans_b=True, m_live=live) if ctx.needs_input_grad[0] else None
        gb = gemm_x6(a, g, trans_a=True, k_live=live) if ctx.needs_input_grad[1] else None
        gc = None
        if ctx.needs_input_grad[2]:
            gc = g.sum(0) if len(ctx.c_shape) == 1 else g
        return ga, gb, gc, None


class _LinearX6(torch.autograd.Function):
    """x @ w^T + bias (nn.Linear: w [N, K]) with regnn_gemm_x6 forward and backward: gx = g w,
    gw = g^T x (w's own layout), gbias = the column sums of g."""

    @staticmethod
    def forward(ctx, x, w, bias):
        if bias is None:
            out = gemm_x6(x, w, trans_b=True)
        else:
            out = bias.expand(x.shape[0], w.shape[0]).contiguous()
            gemm_x6(x, w, trans_b=True, out=out, beta=1.0)
        ctx.save_for_backward(x, w)
        ctx.has_bias = bias is not None
        return out

    @staticmethod
    def backward(ctx, g):
        x, w = ctx.saved_tensors
        g = g.contiguous()
        gx = gemm_x6(g, w) if ctx.needs_input_grad[0] else None
        gw = gemm_x6(g, x, trans_a=True) if ctx.needs_input_grad[1] else None
        gb = g.sum(0) if ctx.has_bias and ctx.needs_input_grad[2] else None
        return gx, gw, gb


class _Copy2d(ctypes.Structure):
    _fields_ = [("src", ctypes.c_void_p), ("dst", ctypes.c_void_p), ("rows", ctypes.c_int64),
                ("cols", ctypes.c_int64), ("s0", ctypes.c_int64), ("s1", ctypes.c_int64)]


def copy_many(dst, src):
    """dst[i].copy_(src[i]) for every pair in one launch (regnn_copy2d_many): fp32 device
    tensors of <= 2 dims, dst contiguous, src any strides (e.g. a transposed weight gradient);
    other pairs take copy_."""
    descs = []
    for d, s_ in zip(dst, src):
        if (d.is_cuda and s_.is_cuda and d.dtype == s_.dtype == torch.float32 and
                d.is_contiguous() and d.numel() == s_.numel() and s_.dim() <= 2 and
                tuple(d.shape) == tuple(s_.shape)):
            if s_.dim() == 2:
                rows, cols, s0, s1 = s_.shape[0], s_.shape[1], s_.stride(0), s_.stride(1)
            elif s_.dim() == 1:
                rows, cols, s0, s1 = 1, s_.shape[0], 0, s_.stride(0)
            else:
                rows, cols, s0, s1 = 1, 1, 0, 0
            descs.append(_Copy2d(s_.data_ptr(), d.data_ptr(), rows, cols, s0, s1))
        else:
            d.copy_(s_)
    if descs:
        arr = (_Copy2d * len(descs))(*descs)
        L.call("regnn_copy2d_many", ctypes.addressof(arr), len(descs), L.stream())


def linear(x, w, bias=None):
    """nn.functional.linear on regnn_gemm_x6 when the operands allow it (else torch)."""
    if (GEMM_X6["mode"] != "off" and x.dim() == 2 and gemm_x6_ok(x, w) and
            (bias is None or (bias.is_cuda and bias.dtype == torch.float32 and bias.dim() == 1))):
        return _LinearX6.apply(x, w, bias)
    return torch.nn.functional.linear(x, w, bias)


# products of at most SMALL_BLAS["macs"] multiply-adds without a live-row bound (the wide NS
# model's layer-1 projection and the [W_c; b_c; 0] W_0 composition: 512-516 x 512 x 512) run on
# hipBLASLt fp32 instead of the x6 GEMM: a few 128 x 128 tiles over a long reduction are
# latency-bound there (split-K partials and a reduce launch); "off": every eligible product on x6
SMALL_BLAS = {"mode": os.environ.get("REGNN_GEMM_SMALL_BLAS", "on"),
              "macs": int(os.environ.get("REGNN_GEMM_SMALL_MACS", str(1 << 28)))}


def mm(a, b, c=None, live=None):
    """c + a @ b on regnn_gemm_x6 when the operands allow it (else torch). live: a one-element
    int32 device tensor with a's live rows (a's rows past it are zero: the GEMMs skip them)."""
    # c: None, a length-N row vector or exactly [M, N] (the x6 epilogue writes M rows with c's
    # row stride; any other broadcastable shape goes to torch)
    M, N = (a.shape[0], b.shape[1]) if a.dim() == 2 and b.dim() == 2 else (-1, -1)
    c_ok = c is None or (c.is_cuda and c.dtype == torch.float32 and
                         (tuple(c.shape) == (N,) or tuple(c.shape) == (M, N)))
    # (not with `live`: a capacity-sized operand's rows past the live count are unspecified, which
    # the x6 kernel skips and hipBLASLt would read)
    small = (SMALL_BLAS["mode"] != "off" and live is None and M > 0 and
             M * N * a.shape[1] <= SMALL_BLAS["macs"])
    if GEMM_X6["mode"] != "off" and gemm_x6_ok(a, b) and c_ok and not small:
        live_ok = (live is not None and live.is_cuda and live.dtype == torch.int32 and
                   live.numel() == 1 and LIVE_ROWS["mode"] != "off")
        return _MMx6.apply(a, b, c, live if live_ok else None)
    return a @ b if c is None else (torch.addmm(c, a, b) if c.dim() <= 2 else c + a @ b)


# ---------------------------------------------------------------------------------------------
# the wide NS model's per-layer epilogue: rs x + bias (+ res) -> LayerNorm -> relu -> dropout
# ---------------------------------------------------------------------------------------------
WIDE_LN_WIDTHS = (64, 128, 256, 512, 1024)


# "on": a live-row count reaches regnn_wide_ln_fwd / _bwd (layer 0 of the wide NS model: ~4.9 k
# live rows of a 13 312-row block at mag-10x); "off": every row formed (A/B)
WIDE_LN_LIVE = {"mode": os.environ.get("REGNN_WIDE_LN_LIVE", "on")}


class _WideLn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, bias, res, gamma, beta, rs, state, layer, p, live):
        n, H = x.shape
        a = torch.empty_like(x)
        y = torch.empty_like(x)
        stats = torch.empty(n, 2, dtype=torch.float32, device=x.device)
        L.call("regnn_wide_ln_fwd", n, H, L.ptr(x), L.ptr(rs), L.ptr(bias), L.ptr(res),
               L.ptr(gamma), L.ptr(beta), L.ptr(state), int(layer), float(p), L.ptr(a),
               L.ptr(stats), L.ptr(y), L.ptr(live), L.stream())
        ctx.save_for_backward(a, stats, rs, gamma, beta, state, live)
        ctx.layer, ctx.p, ctx.has_res = int(layer), float(p), res is not None
        return y

    @staticmethod
    def backward(ctx, gy):
        a, stats, rs, gamma, beta, state, live = ctx.saved_tensors
        n, H = a.shape
        gy = gy.contiguous()
        if gy.data_ptr() % 16:                 # the kernel's float4 rows need 16-byte alignment
            gy = gy.clone()
        gx = torch.empty_like(a)
        gres = torch.empty_like(a) if ctx.has_res and ctx.needs_input_grad[2] else None
        rows = int(L._so.regnn_wide_ln_slab_rows(n, H))
        slab = torch.empty(rows, 3 * H, dtype=torch.float32, device=a.device)
        L.call("regnn_wide_ln_bwd", n, H, L.ptr(gy), L.ptr(a), L.ptr(stats), L.ptr(rs),
               L.ptr(gamma), L.ptr(beta), L.ptr(state), ctx.layer, ctx.p, L.ptr(gx), L.ptr(gres),
               L.ptr(slab), L.ptr(live), L.stream())
        sums = _reduce(slab, 3 * H)
        g_bias, g_gamma, g_beta = sums[:H], sums[H:2 * H], sums[2 * H:]
        return (gx, g_bias, gres, g_gamma, g_beta, None, None, None, None, None)


def wide_ln_ok(x, ln, bias=None):
    return (x.is_cuda and x.dtype == torch.float32 and x.dim() == 2 and x.is_contiguous() and
            x.shape[1] in WIDE_LN_WIDTHS and isinstance(ln, torch.nn.LayerNorm) and
            ln.elementwise_affine and abs(ln.eps - 1e-5) < 1e-12 and x.data_ptr() % 16 == 0 and
            # the kernels read gamma / beta / bias as float4 rows too
            ln.weight.data_ptr() % 16 == 0 and ln.bias.data_ptr() % 16 == 0 and
            _wide_operands_ok(bias))


def _wide_operands_ok(*ts):
    return all(t is None or (t.is_contiguous() and t.data_ptr() % 16 == 0) for t in ts)


def wide_ln_act(x, bias, ln, p=0.0, state=None, layer=0, rs=None, res=None, live=None):
    """dropout(relu(LayerNorm(rs * x + bias + res))) in one launch (regnn_wide_ln_fwd), the
    dropout mask the fused NS step's spec keyed on the sampler `state` and `layer`. live: a
    one-element int32 device count; only rows below it are formed (forward) and differentiated
    (backward) -- for a capacity-sized block whose later rows no consumer reads (their outputs
    and gradients are left unspecified). Not with `res` (its gradient rows would be read)."""
    if p > 0 and state is None:
        raise ValueError("wide_ln_act: dropout needs the sampler state (its mask key)")
    if res is not None:
        res = res.contiguous()
        if res.data_ptr() % 16:
            res = res.clone()
    if not _wide_operands_ok(bias, ln.weight, ln.bias):
        raise ValueError("wide_ln_act: bias / LayerNorm weight and bias must be contiguous and "
                         "16-byte aligned (check wide_ln_ok first)")
    if live is not None and (res is not None or not live.is_cuda or live.dtype != torch.int32 or
                             live.numel() != 1 or WIDE_LN_LIVE["mode"] == "off"):
        live = None
    return _WideLn.apply(x, bias, res, ln.weight, ln.bias,
                         rs, state if p > 0 else None, layer, float(p), live)
