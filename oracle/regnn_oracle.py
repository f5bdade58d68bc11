"""CPU ORACLE for RE-GNN's relation-embedding message-passing hot path — TEST INFRASTRUCTURE.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this
module, and only as the checker / the timed CPU baseline. The product path (``re-gnn_amd``) never
imports it and has no CPU fallback.

What it is: an independent numpy/scipy restatement (float64 by default) of the forward pass AND an
explicit hand-derived backward (VJP) of each layer on the hot path, following the reference source:

* ``REGraphConvOracle``   — layer/REGraphConv.py:52-106
* ``REGATConvOracle``     — layer/REGATConv.py:64-100 (+ DGL ``edge_softmax`` semantics)
* ``REMixHopConvOracle``  — layer/REMixHopConv.py:48-94
* ``RESAGEConvOracle``    — layer/RESAGEConv.py:55-114
* ``REGINConvOracle``     — layer/REGINConv.py:39-66
* ``REGATv2ConvOracle``   — layer/REGATv2Conv.py:103-163
* ``MagREGCNConvOracle``  — mag/regnn_layers.py:80-150 (self_loop_type 2, aggr='mean')
* ``MagREGATConvOracle``  — mag/regnn_layers.py:153-436 (REGATConv / REGATv2Conv, global max)
* model wiring            — model/REGCN.py:35-46, model/REGAT.py:54-66, model/REMixHop.py:87-100
* ``mag_regnn_model``      — mag/regnn_ns.py:216-346 + nll_loss (:404), feats_type 3 and 2

Pinning: every class here is checked against golden vectors produced by running the REFERENCE's own
layer/model source (tests/golden/make_golden.py, on a test-only DGL/PyG shim) — see
tests/test_oracle.py. The DGL/PyG primitive semantics themselves (gspmm sum, edge_softmax,
scatter-mean) come from their documentation: no reference test pins them.

Graph convention (DGL): edge e goes src[e] -> dst[e]; messages flow src -> dst; aggregation is
over the IN-edges of each destination; relation ids are 1-based (``table[rel - 1]``).
"""
import numpy as np
import scipy.sparse as sp

LRELU_SLOPE = 0.01  # nn.LeakyReLU() default, layer/REGraphConv.py:60


# ------------------------------------------------------------------------------------------
# primitives
# ------------------------------------------------------------------------------------------
def lrelu(x, slope=LRELU_SLOPE):
    return np.where(x > 0, x, x * slope)


def lrelu_grad(x, slope=LRELU_SLOPE):
    # torch: d/dx = 1 if x > 0 else slope (slope at exactly 0)
    return np.where(x > 0, 1.0, slope)


def elu(x):
    return np.where(x > 0, x, np.expm1(np.minimum(x, 0)))


def elu_grad(x):
    return np.where(x > 0, 1.0, np.exp(np.minimum(x, 0)))


ACTS = {None: (lambda x: x, lambda x: np.ones_like(x)), "elu": (elu, elu_grad)}


class Graph:
    """src/dst edge lists (DGL order) + cached scipy adjacency (rows = dst, cols = src)."""

    def __init__(self, src, dst, num_nodes, num_dst=None):
        self.src = np.asarray(src, dtype=np.int64)
        self.dst = np.asarray(dst, dtype=np.int64)
        self.n_src = int(num_nodes)
        self.n_dst = int(num_nodes if num_dst is None else num_dst)
        self.E = self.src.size

    def adj(self, w=None, dtype=None):
        """A[v, u] = sum of w over edges u->v (duplicates summed, = DGL gspmm u_mul_e + sum)."""
        if w is None:
            w = np.ones(self.E, dtype=dtype or np.float64)
        w = np.asarray(w, dtype=dtype) if dtype else np.asarray(w)
        return sp.csr_matrix((w, (self.dst, self.src)),
                             shape=(self.n_dst, self.n_src))

    def in_sum(self, w):
        """deg[v] = sum_{e: dst=v} w[e]   (update_all(u_mul_e('nones','ew'), sum))."""
        return np.bincount(self.dst, weights=w, minlength=self.n_dst)

    def out_sum(self, w):
        return np.bincount(self.src, weights=w, minlength=self.n_src)

    def edge_dot(self, a_dst, b_src, chunk=1 << 20):
        """per-edge <a[dst[e]], b[src[e]]> over the trailing axis (SDDMM 'dot'), chunked."""
        out = np.empty((self.E,) + a_dst.shape[1:-1], dtype=np.result_type(a_dst, b_src))
        for s in range(0, self.E, chunk):
            d, u = self.dst[s:s + chunk], self.src[s:s + chunk]
            out[s:s + chunk] = np.einsum("e...f,e...f->e...", a_dst[d], b_src[u])
        return out


def rel_bins(rel, values, R):
    """sum per relation of per-edge values; rel is 1-based. values (E,) or (E,H)."""
    r = np.asarray(rel, dtype=np.int64) - 1
    if values.ndim == 1:
        return np.bincount(r, weights=values, minlength=R)[:, None]
    return np.stack([np.bincount(r, weights=values[:, h], minlength=R)
                     for h in range(values.shape[1])], axis=1)


def degree_norm(g, ew):
    """layer/REGraphConv.py:66-76: norm = clamp(in-degree weighted by ew, min=1)^-1/2."""
    deg = g.in_sum(ew)
    return deg, np.power(np.maximum(deg, 1.0), -0.5)


def degree_norm_vjp(g, deg, g_norm):
    """d norm/d ew[e] for every edge into v. clamp(min=1) passes the gradient where deg >= 1."""
    g_deg = g_norm * (-0.5) * np.power(np.maximum(deg, 1.0), -1.5) * (deg >= 1.0)
    return g_deg[g.dst]


# ------------------------------------------------------------------------------------------
# REGraphConv  (layer/REGraphConv.py:7-106)
# ------------------------------------------------------------------------------------------
class REGraphConvOracle:
    def __init__(self, alpha, in_feats, out_feats, norm=True, activation=None, **_):
        self.alpha, self.fin, self.fout = alpha, in_feats, out_feats
        self.norm, self.act = norm, activation

    def forward(self, g, feat, rel, edge_weight, weight=None, bias=None):
        c = self.c = dict(feat=feat, weight=weight, bias=bias, rel=rel, edge_weight=edge_weight)
        pre_tab = edge_weight * self.alpha                                  # :58
        tab = lrelu(pre_tab)                                                # :60
        ew = tab[np.asarray(rel) - 1, 0]                                    # :61
        c.update(pre_tab=pre_tab, ew=ew)
        x = feat
        if self.norm:
            deg, nrm = degree_norm(g, ew)                                   # :66-75
            c.update(deg=deg, nrm=nrm)
            x = feat * nrm[:, None]                                         # :76
        A = g.adj(ew)
        c["A"] = A
        if self.fin > self.fout:                                            # :78
            if weight is not None:
                x = x @ weight                                              # :81
            c["agg_in"] = x
            rst = A @ x                                                     # :84-86
        else:
            c["agg_in"] = x
            rst = A @ x                                                     # :91-93
            c["agg_out"] = rst
            if weight is not None:
                rst = rst @ weight                                          # :95
        c["pre_norm"] = rst
        if self.norm:
            rst = rst * c["nrm"][:, None]                                   # :98
        if bias is not None:
            rst = rst + bias                                                # :101
        c["pre_act"] = rst
        return ACTS[self.act][0](rst)                                       # :104

    def backward(self, g, gout):
        c = self.c
        grads = {}
        gr = gout * ACTS[self.act][1](c["pre_act"])
        if c["bias"] is not None:
            grads["bias"] = gr.sum(0)
        g_nrm = None
        if self.norm:
            g_nrm = (gr * c["pre_norm"]).sum(1)
            gr = gr * c["nrm"][:, None]
        W, A = c["weight"], c["A"]
        if self.fin > self.fout:
            g_agg_out = gr
        else:
            if W is not None:
                grads["weight"] = c["agg_out"].T @ gr
                g_agg_out = gr @ W.T
            else:
                g_agg_out = gr
        g_agg_in = A.T @ g_agg_out                                          # transposed SpMM
        g_ew = g.edge_dot(g_agg_out, c["agg_in"])                           # SDDMM dot
        if self.fin > self.fout and W is not None:
            x_pre = c["feat"] * c["nrm"][:, None] if self.norm else c["feat"]
            grads["weight"] = x_pre.T @ g_agg_in
            g_x = g_agg_in @ W.T
        else:
            g_x = g_agg_in
        if self.norm:
            g_nrm = g_nrm + (g_x * c["feat"]).sum(1)
            g_feat = g_x * c["nrm"][:, None]
            g_ew = g_ew + degree_norm_vjp(g, c["deg"], g_nrm)
        else:
            g_feat = g_x
        g_tab = rel_bins(c["rel"], g_ew, c["edge_weight"].shape[0])
        grads["edge_weight"] = g_tab * self.alpha * lrelu_grad(c["pre_tab"])
        return g_feat, grads


# ------------------------------------------------------------------------------------------
# REGATConv  (layer/REGATConv.py:10-100)
# ------------------------------------------------------------------------------------------
def edge_softmax(g, z):
    """per-destination softmax over in-edges, max-subtracted (DGL edge_softmax). z (E,H)."""
    H = z.shape[1]
    mx = np.full((g.n_dst, H), -np.inf)
    np.maximum.at(mx, g.dst, z)
    ex = np.exp(z - mx[g.dst])
    s = np.zeros((g.n_dst, H))
    np.add.at(s, g.dst, ex)
    return ex / s[g.dst]


class REGATConvOracle:
    def __init__(self, alpha, in_feats, out_feats, num_heads, negative_slope=0.2,
                 residual=False, activation=None, use_weight=True, edge_feats=True, **_):
        self.alpha, self.fin, self.D, self.H = alpha, in_feats, out_feats, num_heads
        self.slope, self.residual, self.act = negative_slope, residual, activation
        self.use_weight, self.use_ee = use_weight, edge_feats

    def forward(self, g, feat, rel, P):
        """P: dict of reference parameter names -> arrays (fc.weight, attn_l, attn_r,
        edge_weight, res_fc.weight)."""
        N, H, D = feat.shape[0], self.H, self.D
        c = self.c = dict(feat=feat, rel=rel, P=P)
        ft = (feat @ P["fc.weight"].T if self.use_weight else feat).reshape(N, H, D)   # :67
        el = (ft * P["attn_l"]).sum(-1)                                                 # :68
        er = (ft * P["attn_r"]).sum(-1)                                                 # :69
        s = el[g.src] + er[g.dst]                                                       # :80
        if self.use_ee:
            pre_tab = P["edge_weight"] * self.alpha                                     # :72
            c["pre_tab"] = pre_tab
            s = s + lrelu(pre_tab)[np.asarray(rel) - 1]                                 # :74-84
        z = lrelu(s, self.slope)                                                        # :86
        a = edge_softmax(g, z)                                                          # :88
        out = np.zeros((g.n_dst, H, D))
        for h in range(H):
            out[:, h, :] = g.adj(a[:, h]) @ ft[:, h, :]                                  # :90-91
        if self.residual:
            if "res_fc.weight" in P:
                res = (feat @ P["res_fc.weight"].T).reshape(N, -1, D)                   # :94
            else:
                res = feat.reshape(N, -1, D)
            c["res_shape"] = res.shape
            out = out + res
        c.update(ft=ft, s=s, a=a, pre_act=out)
        return ACTS[self.act][0](out)

    def backward(self, g, gout):
        c, P = self.c, self.c["P"]
        feat, ft, a, s = c["feat"], c["ft"], c["a"], c["s"]
        N, H, D = feat.shape[0], self.H, self.D
        grads = {}
        go = gout * ACTS[self.act][1](c["pre_act"])
        g_feat = np.zeros_like(feat)
        if self.residual:
            if "res_fc.weight" in P:
                gr = go.reshape(N, H * D)
                grads["res_fc.weight"] = gr.T @ feat
                g_feat += gr @ P["res_fc.weight"]
            else:
                g_feat += go.sum(1).reshape(N, -1) if c["res_shape"][1] == 1 else go.reshape(N, -1)
        g_ft = np.zeros_like(ft)
        g_a = np.zeros((g.E, H))
        for h in range(H):
            g_ft[:, h, :] = g.adj(a[:, h]).T @ go[:, h, :]
        g_a = g.edge_dot(go, ft)                                        # (E,H)
        t = np.zeros((g.n_dst, H))
        np.add.at(t, g.dst, a * g_a)
        g_z = a * (g_a - t[g.dst])                                      # softmax VJP
        g_s = g_z * lrelu_grad(s, self.slope)
        g_el = np.zeros((N, H))
        np.add.at(g_el, g.src, g_s)
        g_er = np.zeros((N, H))
        np.add.at(g_er, g.dst, g_s)
        if self.use_ee:
            g_tab = rel_bins(c["rel"], g_s, P["edge_weight"].shape[0])
            grads["edge_weight"] = g_tab * self.alpha * lrelu_grad(c["pre_tab"])
        g_ft += g_el[..., None] * P["attn_l"] + g_er[..., None] * P["attn_r"]
        grads["attn_l"] = (g_el[..., None] * ft).sum(0, keepdims=True)
        grads["attn_r"] = (g_er[..., None] * ft).sum(0, keepdims=True)
        gf = g_ft.reshape(N, H * D)
        if self.use_weight:
            grads["fc.weight"] = gf.T @ feat
            g_feat += gf @ P["fc.weight"]
        else:
            g_feat += gf
        return g_feat, grads


# ------------------------------------------------------------------------------------------
# REMixHopConv  (layer/REMixHopConv.py:7-94)
# ------------------------------------------------------------------------------------------
class REMixHopConvOracle:
    def __init__(self, alpha, in_feats, out_feats, p=(0, 1, 2), activation=None, **_):
        self.alpha, self.p, self.act = alpha, list(p), activation

    def forward(self, g, feats, rel, P):
        c = self.c = dict(rel=rel, P=P)
        pre_tab = P["edge_weight"] * self.alpha
        ew = lrelu(pre_tab)[np.asarray(rel) - 1, 0]                         # :50-55
        deg, nrm = degree_norm(g, ew)                                       # :58-64
        A1 = g.adj(None)                                                    # copy_u: unweighted
        fs, outs = [feats], []
        for j in range(max(self.p) + 1):                                    # :72
            if j in self.p:
                outs.append(fs[-1] @ P[f"weights.{j}.weight"].T)            # :74-76
            if j < max(self.p):   # the last propagate (:78-82) feeds nothing: skipped
                fs.append(nrm[:, None] * (A1 @ (nrm[:, None] * fs[-1])))
        final = np.concatenate(outs, axis=1)                                # :84
        c.update(pre_tab=pre_tab, deg=deg, nrm=nrm, A1=A1, fs=fs, pre_act=final)
        return ACTS[self.act][0](final)                                     # :88-90

    def backward(self, g, gout):
        c, P = self.c, self.c["P"]
        nrm, A1, fs = c["nrm"][:, None], c["A1"], c["fs"]
        gf_all = gout * ACTS[self.act][1](c["pre_act"])
        grads = {}
        width = gf_all.shape[1] // len(self.p)
        g_f = [np.zeros_like(f) for f in fs]
        for k, j in enumerate(self.p):
            go = gf_all[:, k * width:(k + 1) * width]
            grads[f"weights.{j}.weight"] = go.T @ fs[j]
            g_f[j] += go @ P[f"weights.{j}.weight"]
        g_nrm = np.zeros(nrm.shape[0])
        for j in range(len(fs) - 1, 0, -1):     # f_j = nrm * A1 (nrm * f_{j-1})
            gy = g_f[j]
            t = A1 @ (nrm * fs[j - 1])
            back = A1.T @ (nrm * gy)
            g_nrm += (gy * t).sum(1) + (fs[j - 1] * back).sum(1)
            g_f[j - 1] += nrm * back
        g_ew = degree_norm_vjp(g, c["deg"], g_nrm)
        g_tab = rel_bins(c["rel"], g_ew, P["edge_weight"].shape[0])
        grads["edge_weight"] = g_tab * self.alpha * lrelu_grad(c["pre_tab"])
        return g_f[0], grads


# ------------------------------------------------------------------------------------------
# RESAGEConv / REGINConv (layer/RESAGEConv.py:55-114, layer/REGINConv.py:39-66): deg^-1 norm
# ------------------------------------------------------------------------------------------
def degree_norm_pow(g, ew, power):
    deg = g.in_sum(ew)
    return deg, np.power(np.maximum(deg, 1.0), power)


def degree_norm_pow_vjp(g, deg, g_norm, power):
    g_deg = g_norm * power * np.power(np.maximum(deg, 1.0), power - 1.0) * (deg >= 1.0)
    return g_deg[g.dst]


class RESAGEConvOracle:
    """deg^-1 pre-norm of the aggregated features, no post-norm, root term feat @ weight (the
    reference's forward uses ``self.weight`` for the root, :60-61; ``weight_root`` is unused)."""

    def __init__(self, alpha, in_feats, out_feats, norm=True, activation=None, **_):
        self.alpha, self.fin, self.fout = alpha, in_feats, out_feats
        self.norm, self.act = norm, activation

    def forward(self, g, feat, rel, P):
        W, b = P.get("weight"), P.get("bias")
        c = self.c = dict(feat=feat, rel=rel, P=P)
        pre_tab = P["edge_weight"] * self.alpha                             # :65
        ew = lrelu(pre_tab)[np.asarray(rel) - 1, 0]                         # :67-68
        root = feat @ W if W is not None else feat                          # :60-63
        x = feat
        if self.norm:
            deg, nrm = degree_norm_pow(g, ew, -1.0)                         # :73-80
            c.update(deg=deg, nrm=nrm)
            x = feat * nrm[:, None]                                         # :83
        A = g.adj(ew)
        if self.fin > self.fout:                                            # :85
            agg_in = x @ W if W is not None else x                          # :88
            rst = A @ agg_in
        else:
            agg_in = x
            rst = A @ x                                                     # :98-101
            c["agg_out"] = rst
            if W is not None:
                rst = rst @ W                                               # :103
        rst = rst + root                                                    # :109
        if b is not None:
            rst = rst + b                                                   # :112
        c.update(pre_tab=pre_tab, A=A, x=x, agg_in=agg_in, pre_act=rst)
        return ACTS[self.act][0](rst)

    def backward(self, g, gout):
        c, P = self.c, self.c["P"]
        W, A, feat = P.get("weight"), c["A"], c["feat"]
        grads = {}
        gr = gout * ACTS[self.act][1](c["pre_act"])
        if P.get("bias") is not None:
            grads["bias"] = gr.sum(0)
        if W is not None:
            grads["weight"] = feat.T @ gr
            g_feat = gr @ W.T
        else:
            g_feat = gr.copy()
        if self.fin > self.fout:
            g_agg_in = A.T @ gr
            g_ew = g.edge_dot(gr, c["agg_in"])
            if W is not None:
                grads["weight"] = grads["weight"] + c["x"].T @ g_agg_in
                g_x = g_agg_in @ W.T
            else:
                g_x = g_agg_in
        else:
            if W is not None:
                grads["weight"] = grads["weight"] + c["agg_out"].T @ gr
                g_out = gr @ W.T
            else:
                g_out = gr
            g_x = A.T @ g_out
            g_ew = g.edge_dot(g_out, c["x"])
        if self.norm:
            g_nrm = (g_x * feat).sum(1)
            g_feat = g_feat + g_x * c["nrm"][:, None]
            g_ew = g_ew + degree_norm_pow_vjp(g, c["deg"], g_nrm, -1.0)
        else:
            g_feat = g_feat + g_x
        g_tab = rel_bins(c["rel"], g_ew, P["edge_weight"].shape[0])
        grads["edge_weight"] = g_tab * self.alpha * lrelu_grad(c["pre_tab"])
        return g_feat, grads


class REGINConvOracle:
    """rst = deg^-1 * sum ew * feat[u], then apply_func (a Linear here) and activation. The
    reference always reduces with sum whatever ``aggregator_type`` says (``_reducer`` unused)."""

    def __init__(self, alpha, apply_linear=None, activation=None, **_):
        self.alpha, self.lin, self.act = alpha, apply_linear, activation

    def forward(self, g, feat, rel, P):
        c = self.c = dict(feat=feat, rel=rel, P=P)
        pre_tab = P["edge_weight"] * self.alpha                             # :42-44
        ew = lrelu(pre_tab)[np.asarray(rel) - 1, 0]                         # :45
        deg, nrm = degree_norm_pow(g, ew, -1.0)                             # :48-54
        A = g.adj(ew)
        agg = A @ feat                                                      # :58-60
        rst = agg * nrm[:, None]                                            # :62
        c.update(pre_tab=pre_tab, deg=deg, nrm=nrm, A=A, agg=agg, rst=rst)
        if self.lin:
            rst = rst @ P["apply_func.weight"].T + P["apply_func.bias"]      # :63-64
        c["pre_act"] = rst
        return ACTS[self.act][0](rst)

    def backward(self, g, gout):
        c, P = self.c, self.c["P"]
        grads = {}
        gr = gout * ACTS[self.act][1](c["pre_act"])
        if self.lin:
            grads["apply_func.weight"] = gr.T @ c["rst"]
            grads["apply_func.bias"] = gr.sum(0)
            gr = gr @ P["apply_func.weight"]
        g_nrm = (gr * c["agg"]).sum(1)
        g_agg = gr * c["nrm"][:, None]
        g_feat = c["A"].T @ g_agg
        g_ew = g.edge_dot(g_agg, c["feat"]) + degree_norm_pow_vjp(g, c["deg"], g_nrm, -1.0)
        g_tab = rel_bins(c["rel"], g_ew, P["edge_weight"].shape[0])
        grads["edge_weight"] = g_tab * self.alpha * lrelu_grad(c["pre_tab"])
        return g_feat, grads


# ------------------------------------------------------------------------------------------
# REGATv2Conv (layer/REGATv2Conv.py:103-163): score = attn . LeakyReLU(fs[u] + fd[v])
# ------------------------------------------------------------------------------------------
class REGATv2ConvOracle:
    def __init__(self, alpha, in_feats, out_feats, num_heads, negative_slope=0.2,
                 residual=False, activation=None, share_weights=False, edge_feats=True, **_):
        self.alpha, self.fin, self.D, self.H = alpha, in_feats, out_feats, num_heads
        self.slope, self.residual, self.act = negative_slope, residual, activation
        self.share, self.use_ee = share_weights, edge_feats

    def forward(self, g, feat, rel, P):
        N, H, D = feat.shape[0], self.H, self.D
        c = self.c = dict(feat=feat, rel=rel, P=P)
        fs = (feat @ P["fc_src.weight"].T + P["fc_src.bias"]).reshape(N, H, D)   # :127-129
        if self.share:
            fd = fs                                                             # :131
        else:
            fd = (feat @ P["fc_dst.weight"].T + P["fc_dst.bias"]).reshape(N, H, D)  # :133-134
        pre = fs[g.src] + fd[g.dst]                                             # :139
        z = lrelu(pre, self.slope)                                              # :140
        e = (z * P["attn"]).sum(-1)                                             # :141
        if self.use_ee:
            pre_tab = P["edge_weight"] * self.alpha                             # :144
            c["pre_tab"] = pre_tab
            e = e + lrelu(pre_tab)[np.asarray(rel) - 1]                         # :146-149
        a = edge_softmax(g, e)                                                  # :152
        out = np.zeros((g.n_dst, H, D))
        for h in range(H):
            out[:, h, :] = g.adj(a[:, h]) @ fs[:, h, :]                         # :154-156
        if self.residual:
            if "res_fc.weight" in P:
                res = (feat @ P["res_fc.weight"].T + P["res_fc.bias"]).reshape(N, -1, D)
            else:
                res = feat.reshape(N, -1, D)                                    # Identity
            c["res_shape"] = res.shape
            out = out + res                                                     # :158-160
        c.update(fs=fs, pre=pre, z=z, a=a, pre_act=out)
        return ACTS[self.act][0](out)

    def backward(self, g, gout):
        c, P = self.c, self.c["P"]
        feat, fs, a, pre, z = c["feat"], c["fs"], c["a"], c["pre"], c["z"]
        N, H, D = feat.shape[0], self.H, self.D
        grads = {}
        go = gout * ACTS[self.act][1](c["pre_act"])
        g_feat = np.zeros_like(feat)
        if self.residual:
            if "res_fc.weight" in P:
                gr = go.reshape(N, H * D)
                grads["res_fc.weight"] = gr.T @ feat
                grads["res_fc.bias"] = gr.sum(0)
                g_feat += gr @ P["res_fc.weight"]
            else:
                g_feat += go.sum(1).reshape(N, -1) if c["res_shape"][1] == 1 else go.reshape(N, -1)
        g_fs = np.zeros_like(fs)
        for h in range(H):
            g_fs[:, h, :] = g.adj(a[:, h]).T @ go[:, h, :]
        g_a = g.edge_dot(go, fs)                                                # (E,H)
        t = np.zeros((g.n_dst, H))
        np.add.at(t, g.dst, a * g_a)
        g_e = a * (g_a - t[g.dst])                                              # softmax VJP
        if self.use_ee:
            g_tab = rel_bins(c["rel"], g_e, P["edge_weight"].shape[0])
            grads["edge_weight"] = g_tab * self.alpha * lrelu_grad(c["pre_tab"])
        grads["attn"] = (g_e[..., None] * z).sum(0, keepdims=True)
        g_pre = g_e[..., None] * P["attn"] * lrelu_grad(pre, self.slope)        # (E,H,D)
        np.add.at(g_fs, g.src, g_pre)
        g_fd = np.zeros_like(fs)
        np.add.at(g_fd, g.dst, g_pre)
        if self.share:
            g_fs = g_fs + g_fd
        gfs = g_fs.reshape(N, H * D)
        grads["fc_src.weight"] = gfs.T @ feat
        grads["fc_src.bias"] = gfs.sum(0)
        g_feat += gfs @ P["fc_src.weight"]
        if not self.share:
            gfd = g_fd.reshape(N, H * D)
            grads["fc_dst.weight"] = gfd.T @ feat
            grads["fc_dst.bias"] = gfd.sum(0)
            g_feat += gfd @ P["fc_dst.weight"]
        return g_feat, grads


# ------------------------------------------------------------------------------------------
# mag REGCNConv  (mag/regnn_layers.py:24-150), self_loop_type == 2, aggr='mean'
# ------------------------------------------------------------------------------------------
def layer_norm(x, w, b, eps=1e-5):
    mu = x.mean(1, keepdims=True)
    var = x.var(1, keepdims=True)
    rstd = 1.0 / np.sqrt(var + eps)
    xh = (x - mu) * rstd
    return xh * w + b, (xh, rstd)


def layer_norm_vjp(g, w, cache):
    xh, rstd = cache
    gxh = g * w
    gx = rstd * (gxh - gxh.mean(1, keepdims=True) - xh * (gxh * xh).mean(1, keepdims=True))
    return gx, (g * xh).sum(0), g.sum(0)


class MagREGCNConvOracle:
    def __init__(self, n_dst, num_edge_types, scaling_factor, residual=False, use_norm="ln", **_):
        self.n_dst, self.net = n_dst, num_edge_types
        self.alpha, self.residual, self.use_norm = scaling_factor, residual, use_norm

    def block(self, src, dst, edge_type, target_node_type, n_src):
        """append target self loops typed ntype + num_edge_types (mag/regnn_layers.py:90-96)."""
        loop = np.arange(self.n_dst)
        s = np.concatenate([src, loop])
        d = np.concatenate([dst, loop])
        t = np.concatenate([edge_type, np.asarray(target_node_type) + self.net])
        return Graph(s, d, n_src, num_dst=self.n_dst), t

    def forward(self, x, src, dst, edge_type, target_node_type, P):
        g, et = self.block(src, dst, edge_type, target_node_type, x.shape[0])
        W = P["weight"]
        xs = x @ W                                                          # :102
        xt = x[:self.n_dst] @ W                                             # :104/106
        pre_tab = P["relation_weight"] * self.alpha                         # :110
        ew = lrelu(pre_tab)[et]                                             # :111-113 (one-hot)
        cnt = np.maximum(np.bincount(g.dst, minlength=self.n_dst), 1).astype(np.float64)
        agg = (g.adj(ew) @ xs) / cnt[:, None]                               # aggr='mean' :129
        out = agg + P["bias"]                                               # update() :148
        if self.residual:
            out = out + xt                                                  # :131-132
        ln = None
        if self.use_norm == "ln":
            out, ln = layer_norm(out, P["norm.weight"], P["norm.bias"])     # :134-135
        self.c = dict(g=g, et=et, x=x, xs=xs, ew=ew, cnt=cnt, pre_tab=pre_tab, ln=ln, P=P)
        return out

    def edge_weights(self, use_softmax):
        """return_weights' ew of the last forward (mag/regnn_layers.py:116-126,137): softmax of
        the relation weights over each target's in-edges with ONE global max subtracted and
        + 1e-16 in the denominator (mag/utils.py:45-57), else weight / weighted in-degree
        (mag/utils.py:15-21). Edge order: sampled edges, then the appended self loops."""
        c = self.c
        w, col = c["ew"], c["g"].dst
        if use_softmax:
            e = np.exp(w - w.max())
            den = np.bincount(col, weights=e, minlength=self.n_dst)
            return e / (den[col] + 1e-16)
        deg = np.bincount(col, weights=w, minlength=self.n_dst)
        return w / deg[col]

    def backward(self, gout):
        c, P = self.c, self.c["P"]
        g, W = c["g"], P["weight"]
        grads = {}
        if self.use_norm == "ln":
            gout, grads["norm.weight"], grads["norm.bias"] = layer_norm_vjp(
                gout, P["norm.weight"], c["ln"])
        grads["bias"] = gout.sum(0)
        gm = gout / c["cnt"][:, None]
        g_xs = g.adj(c["ew"]).T @ gm
        g_ew = g.edge_dot(gm, c["xs"])
        R = P["relation_weight"].shape[0]
        g_tab = np.bincount(c["et"], weights=g_ew, minlength=R)
        grads["relation_weight"] = g_tab * self.alpha * lrelu_grad(c["pre_tab"])
        x = c["x"]
        gW = x.T @ g_xs
        g_x = g_xs @ W.T
        if self.residual:
            gW += x[:self.n_dst].T @ gout
            g_x[:self.n_dst] += gout @ W.T
        grads["weight"] = gW
        return g_x, grads


class MagREGATConvOracle:
    """mag/regnn_layers.py:153-315 (v2=False) and :318-436 REGATv2Conv (v2=True), self_loop_type
    2, concat heads: the edge softmax subtracts ONE global max and adds 1e-16 (mag/utils.py:45-57).
    The backward ignores the max's own gradient (exactly 0 up to the 1e-16 term)."""

    def __init__(self, n_dst, num_edge_types, scaling_factor, heads, out_channels, v2=False,
                 residual=False, use_norm="ln", negative_slope=0.2, **_):
        self.n_dst, self.net, self.alpha = n_dst, num_edge_types, scaling_factor
        self.H, self.C, self.v2 = heads, out_channels, v2
        self.residual, self.use_norm, self.slope = residual, use_norm, negative_slope

    def forward(self, x, src, dst, edge_type, target_node_type, P):
        H, C, nd = self.H, self.C, self.n_dst
        g, et = MagREGCNConvOracle(nd, self.net, self.alpha).block(src, dst, edge_type,
                                                                   target_node_type, x.shape[0])
        Wl = P["lin_src.weight"]
        xs = (x @ Wl.T).reshape(-1, H, C)                                   # :267-272
        xd = (x[:nd] @ Wl.T).reshape(-1, H, C)
        pre_tab = P["relation_weight"] * self.alpha                         # :294
        tab = lrelu(pre_tab)                                                # :295
        c = self.c = dict(g=g, et=et, x=x, xs=xs, xd=xd, pre_tab=pre_tab, P=P)
        if self.v2:
            pre = xs[g.src] + xd[g.dst]                                     # :399-401
            zz = lrelu(pre, self.slope)                                     # :403
            z = (zz * P["att"]).sum(-1) + tab[et]                           # :404-413
            c.update(pre=pre, zz=zz)
        else:
            a_s = (xs * P["att_src"]).sum(-1)                               # :289
            a_d = (xd * P["att_dst"]).sum(-1)                               # :290
            s = tab[et] + a_s[g.src] + a_d[g.dst]                           # :298-304
            z = lrelu(s, self.slope)                                        # :305
            c["s"] = s
        ex = np.exp(z - z.max())                                            # utils.py:52-53
        S = np.zeros((nd, H))
        np.add.at(S, g.dst, ex)
        a = ex / (S[g.dst] + 1e-16)                                         # utils.py:57
        out = np.zeros((nd, H, C))
        for h in range(H):
            out[:, h, :] = g.adj(a[:, h]) @ xs[:, h, :]                     # propagate :312
        out = out.reshape(nd, H * C) + P["bias"]                            # :314-319
        if self.residual:
            out = out + xd.reshape(nd, H * C)                               # :321-322
        ln = None
        if self.use_norm == "ln":
            out, ln = layer_norm(out, P["norm.weight"], P["norm.bias"])     # :324-325
        c.update(a=a, ln=ln)
        return out

    def backward(self, gout):
        c, P = self.c, self.c["P"]
        g, xs, xd, a, x = c["g"], c["xs"], c["xd"], c["a"], c["x"]
        H, C, nd = self.H, self.C, self.n_dst
        grads = {}
        if self.use_norm == "ln":
            gout, grads["norm.weight"], grads["norm.bias"] = layer_norm_vjp(
                gout, P["norm.weight"], c["ln"])
        grads["bias"] = gout.sum(0)
        g3 = gout.reshape(nd, H, C)
        g_xd = g3.copy() if self.residual else np.zeros_like(xd)
        g_xs = np.zeros_like(xs)
        for h in range(H):
            g_xs[:, h, :] = g.adj(a[:, h]).T @ g3[:, h, :]
        g_a = g.edge_dot(g3, xs)                                            # (E, H)
        t = np.zeros((nd, H))
        np.add.at(t, g.dst, a * g_a)
        g_z = a * (g_a - t[g.dst])                                          # softmax VJP
        R = P["relation_weight"].shape[0]
        if self.v2:
            g_tab = np.stack([np.bincount(c["et"], weights=g_z[:, h], minlength=R)
                              for h in range(H)], 1)
            grads["att"] = (g_z[..., None] * c["zz"]).sum(0, keepdims=True)
            g_pre = g_z[..., None] * P["att"] * lrelu_grad(c["pre"], self.slope)
            np.add.at(g_xs, g.src, g_pre)
            np.add.at(g_xd, g.dst, g_pre)
        else:
            g_s = g_z * lrelu_grad(c["s"], self.slope)
            g_tab = np.stack([np.bincount(c["et"], weights=g_s[:, h], minlength=R)
                              for h in range(H)], 1)
            g_as = np.zeros((xs.shape[0], H))
            np.add.at(g_as, g.src, g_s)
            g_ad = np.zeros((nd, H))
            np.add.at(g_ad, g.dst, g_s)
            grads["att_src"] = (g_as[..., None] * xs).sum(0, keepdims=True)
            grads["att_dst"] = (g_ad[..., None] * xd).sum(0, keepdims=True)
            g_xs += g_as[..., None] * P["att_src"]
            g_xd += g_ad[..., None] * P["att_dst"]
        grads["relation_weight"] = g_tab * self.alpha * lrelu_grad(c["pre_tab"])
        Wl = P["lin_src.weight"]
        gs2, gd2 = g_xs.reshape(-1, H * C), g_xd.reshape(nd, H * C)
        grads["lin_src.weight"] = gs2.T @ x + gd2.T @ x[:nd]
        g_x = gs2 @ Wl
        g_x[:nd] += gd2 @ Wl
        return g_x, grads


# ------------------------------------------------------------------------------------------
# model wiring (eval mode: dropout = identity)
# ------------------------------------------------------------------------------------------
class Linear:
    def __init__(self, W, b=None):
        self.W, self.b = W, b

    def forward(self, x):
        self.x = x
        y = x @ self.W.T
        return y + self.b if self.b is not None else y

    def backward(self, g):
        gr = {"weight": g.T @ self.x}
        if self.b is not None:
            gr["bias"] = g.sum(0)
        return g @ self.W, gr


def _input_proj(P, feats):
    lins = [Linear(P[f"fc_list.{i}.weight"], P[f"fc_list.{i}.bias"]) for i in range(len(feats))]
    return lins, np.concatenate([l.forward(f) for l, f in zip(lins, feats)], 0)


def _input_proj_vjp(lins, feats, g, grads):
    o = 0
    for i, (l, f) in enumerate(zip(lins, feats)):
        _, gr = l.backward(g[o:o + f.shape[0]])
        o += f.shape[0]
        grads[f"fc_list.{i}.weight"], grads[f"fc_list.{i}.bias"] = gr["weight"], gr["bias"]


def regcn_model(g, feats, rel, P, num_layers, alpha, gout):
    """model/REGCN.py:6-46 forward + VJP. Returns logits, embeddings, grads."""
    lins, h = _input_proj(P, feats)
    layers = []
    for l in range(num_layers):
        mid = 0 < l < num_layers - 1
        layers.append(REGraphConvOracle(alpha, h.shape[1], h.shape[1], norm=True,
                                        activation="elu" if mid else None))
        h = layers[-1].forward(g, h, rel, P[f"layers.{l}.edge_weight"],
                               P.get(f"layers.{l}.weight"), P.get(f"layers.{l}.bias"))
    out_lin = Linear(P["out_lin.weight"], P["out_lin.bias"])
    logits = out_lin.forward(h)
    grads = {}
    gh, gr = out_lin.backward(gout)
    grads["out_lin.weight"], grads["out_lin.bias"] = gr["weight"], gr["bias"]
    for l in range(num_layers - 1, -1, -1):
        gh, gr = layers[l].backward(g, gh)
        for k, v in gr.items():
            grads[f"layers.{l}.{k}"] = v
    _input_proj_vjp(lins, feats, gh, grads)
    return logits, h, grads


def regat_model(g, feats, rel, P, num_layers, heads, hidden, alpha, gout, slope=0.01):
    """model/REGAT.py:6-66: per-type Linear, L GAT layers (ELU), last layer applied TWICE."""
    lins, h = _input_proj(P, feats)

    def params(l):
        pre = f"gat_layers.{l}."
        return {k[len(pre):]: v for k, v in P.items() if k.startswith(pre)}

    def make(l, width):
        if l < num_layers - 1:   # input / hidden layers: fc + ELU (model/REGAT.py:84-92)
            return REGATConvOracle(alpha, width, hidden, heads[l], slope, residual=False,
                                   activation="elu", use_weight=True)
        # output layer: Identity fc, no activation, heads[-2] (model/REGAT.py:94-97)
        return REGATConvOracle(alpha, width, hidden, heads[-2], slope, residual=False,
                               activation=None, use_weight=False)

    calls = []
    seq = list(range(num_layers)) + [num_layers - 1]   # last layer applied twice (:61-64)
    for i, l in enumerate(seq):
        o = make(l, h.shape[1])
        y = o.forward(g, h, rel, params(l))
        calls.append((l, o))
        h = y.reshape(h.shape[0], -1) if i < len(seq) - 1 else y
    emb = h
    out_lin = Linear(P["out_lin.weight"], P["out_lin.bias"])
    logits = out_lin.forward(emb.reshape(emb.shape[0], -1))
    grads = {}
    gh, gr = out_lin.backward(gout)
    grads["out_lin.weight"], grads["out_lin.bias"] = gr["weight"], gr["bias"]
    for l, o in reversed(calls):
        gh, gr = o.backward(g, gh.reshape(gh.shape[0], o.H, o.D))
        for k, v in gr.items():
            key = f"gat_layers.{l}.{k}"
            grads[key] = grads.get(key, 0) + v
        gh = gh.reshape(gh.shape[0], -1)
    _input_proj_vjp(lins, feats, gh, grads)
    return logits, emb.mean(1), grads


def remixhop_model(g, feats, rel, P, num_layers, hidden, alpha, gout, p=(0, 1, 2)):
    """model/REMixHop.py:19-100 (activation ELU, no batchnorm, dropout 0)."""
    lins, h = _input_proj(P, feats)
    layers = []
    for l in range(num_layers):
        o = REMixHopConvOracle(alpha, h.shape[1], hidden, p=p, activation="elu")
        pl = {k[len(f"layers.{l}."):]: v for k, v in P.items() if k.startswith(f"layers.{l}.")}
        h = o.forward(g, h, rel, pl)
        layers.append(o)
    fc = Linear(P["fc_layers.weight"])
    logits = fc.forward(h)
    grads = {}
    gh, gr = fc.backward(gout)
    grads["fc_layers.weight"] = gr["weight"]
    for l in range(num_layers - 1, -1, -1):
        gh, gr = layers[l].backward(g, gh)
        for k, v in gr.items():
            grads[f"layers.{l}.{k}"] = v
    _input_proj_vjp(lins, feats, gh, grads)
    return logits, h, grads


# ------------------------------------------------------------------------------------------
# mag REGNN (mag/regnn_ns.py:216-346) + nll_loss (:404), eval mode, on a sampled batch
# ------------------------------------------------------------------------------------------
def mag_regnn_model(x_dict, node_type, local, n_id, adjs, edge_type, P, y, feats_type=3,
                    num_edge_types=7, alpha=10.0, target_node_type=0, residual=False):
    """forward + VJP of the reference REGNN for model 'regcn', self_loop_type 2, LayerNorm.
    adjs: [(src_local, dst_local, e_id, (n_src, n_dst))] outermost hop first (PyG order).
    Returns (log-probabilities, mean nll loss, {parameter name: gradient})."""
    nid = np.asarray(n_id)
    nt, loc = np.asarray(node_type)[nid], np.asarray(local)[nid]
    grads = {}
    if feats_type == 2:                                              # regnn_ns.py:306-315
        t = np.zeros((nid.size, P["lin.weight"].shape[1]))
        for key, x in x_dict.items():
            m = nt == key
            t[m] = x[loc[m]]
        for key in {int(k.split(".")[1]) for k in P if k.startswith("emb_dict.")}:
            m = nt == key
            t[m] = P[f"emb_dict.{key}"][loc[m]]
        lin = Linear(P["lin.weight"], P["lin.bias"])
        h = lin.forward(t)
    else:                                                            # regnn_ns.py:316-324
        h = np.zeros((nid.size, P["lins.0.weight"].shape[0]))
        lins = {}
        for key, x in x_dict.items():
            m = nt == key
            lins[key] = Linear(P[f"lins.{key}.weight"], P[f"lins.{key}.bias"])
            h[m] = lins[key].forward(x[loc[m]])
    et = np.asarray(edge_type)
    caches, x, ntype = [], h, nt
    for i, (s_, d_, e_, size) in enumerate(adjs):                    # regnn_ns.py:335-343
        ntype = ntype[:size[1]]
        pc = {k[len(f"convs.{i}."):]: v for k, v in P.items() if k.startswith(f"convs.{i}.")}
        o = MagREGCNConvOracle(size[1], num_edge_types, alpha, residual=residual, use_norm="ln")
        yv = o.forward(x, np.asarray(s_), np.asarray(d_), et[np.asarray(e_)], ntype, pc)
        caches.append((o, yv))
        x = np.maximum(yv, 0)
    out_lin = Linear(P["out_lin.weight"], P["out_lin.bias"])
    z = out_lin.forward(x)
    zmax = z.max(1, keepdims=True)
    logp = z - (zmax + np.log(np.exp(z - zmax).sum(1, keepdims=True)))
    yb = np.asarray(y)
    n = yb.size
    loss = -logp[np.arange(n), yb].mean()
    g = np.zeros_like(logp)
    g[np.arange(n), yb] = -1.0 / n                                   # nll_loss mean
    gz = g - np.exp(logp) * g.sum(1, keepdims=True)                  # log_softmax VJP
    gx, gr = out_lin.backward(gz)
    grads["out_lin.weight"], grads["out_lin.bias"] = gr["weight"], gr["bias"]
    for i in range(len(caches) - 1, -1, -1):
        o, yv = caches[i]
        gx, grc = o.backward(gx * (yv > 0))
        for k, v in grc.items():
            grads[f"convs.{i}.{k}"] = v
    if feats_type == 2:
        gt, gr = lin.backward(gx)
        grads["lin.weight"], grads["lin.bias"] = gr["weight"], gr["bias"]
        for key in {int(k.split(".")[1]) for k in P if k.startswith("emb_dict.")}:
            m = nt == key
            ge = np.zeros_like(P[f"emb_dict.{key}"])
            np.add.at(ge, loc[m], gt[m])
            grads[f"emb_dict.{key}"] = ge
    else:
        for key, l_ in lins.items():
            m = nt == key
            _, gr = l_.backward(gx[m])
            grads[f"lins.{key}.weight"], grads[f"lins.{key}.bias"] = gr["weight"], gr["bias"]
    return logp, loss, grads


# ------------------------------------------------------------------------------------------
# fused-dropout mask of regnn_spmm_fwd_dropout (this build's spec, include/regnn_hip.h)
# ------------------------------------------------------------------------------------------
def _fmix32(h):
    h = np.asarray(h, dtype=np.uint32)
    with np.errstate(over="ignore"):
        h = h ^ (h >> np.uint32(16))
        h = h * np.uint32(0x85EBCA6B)
        h = h ^ (h >> np.uint32(13))
        h = h * np.uint32(0xC2B2AE35)
        h = h ^ (h >> np.uint32(16))
    return h


def dropout_mask(seed, rows, F, ev, keep16):
    """0/1 keep mask [rows, F] of the fused dropout for a 64-bit seed (ev = features per 16-byte
    vector: 4 fp32, 8 bf16)."""
    seed = int(seed) & ((1 << 64) - 1)
    lo, hi = np.uint32(seed & 0xFFFFFFFF), np.uint32(seed >> 32)
    key = _fmix32(lo ^ _fmix32(hi ^ np.uint32(0x5BD1E995)))
    nvec = F // ev
    c = (np.arange(rows, dtype=np.uint64)[:, None] * np.uint64(nvec)
         + np.arange(nvec, dtype=np.uint64)[None, :])
    hi = (c >> np.uint64(32)).astype(np.uint32)
    bits = 8 if keep16 % 256 == 0 else 16
    per = 32 // bits
    with np.errstate(over="ignore"):
        h = _fmix32((c & np.uint64(0xFFFFFFFF)).astype(np.uint32) ^ key
                    ^ ((hi << np.uint32(16)) | (hi >> np.uint32(16))))
        keep = np.empty((rows, nvec, ev), dtype=bool)
        lim = np.uint32(keep16 >> 8) if bits == 8 else np.uint32(keep16)
        mask = np.uint32((1 << bits) - 1)
        for k in range(ev // per):
            if k:
                h = _fmix32(h + np.uint32(0x9E3779B9))
            for b in range(per):
                keep[:, :, per * k + b] = ((h >> np.uint32(bits * b)) & mask) < lim
    return keep.reshape(rows, F).astype(np.float64)
