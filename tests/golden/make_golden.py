"""Generate the golden vectors in tests/golden/*.npz by running the REFERENCE's own layer/model
source (imported read-only from /root/reference) on a test-only pure-torch DGL/PyG shim
(tests/golden/refshim), in float64 on the CPU of this container.

This script is the ONLY place the reference is executed. It needs /root/reference and is never
run on the GPU box (it is listed in .gpurunignore); the fixtures it writes are plain data
(inputs + expected outputs + expected gradients) and travel with the repo.

Run:  python tests/golden/make_golden.py        (writes tests/golden/*.npz)

Every input is drawn in float32 and widened, so the fp32 GPU path consumes bit-identical inputs;
outputs and gradients are computed in float64 and stored rounded to float32.
"""
import importlib
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
SHIM = os.path.join(HERE, "refshim")


def _purge(prefixes):
    for name in list(sys.modules):
        if any(name == p or name.startswith(p + ".") for p in prefixes):
            del sys.modules[name]


def _use_paths(paths):
    for p in reversed(paths):
        if p in sys.path:
            sys.path.remove(p)
        sys.path.insert(0, p)


# ------------------------------------------------------------------------------------------
# small seeded multi-relation graphs
# ------------------------------------------------------------------------------------------
def make_hetero_graph(rng, type_counts, n_edges, n_dup=10, isolate=5):
    """Random typed directed graph WITHOUT self loops, then self loops appended (DGL order).

    Relation id of a non-loop edge = 1 + index of its (src type, dst type) pair among the pairs
    present; self loop of a node of type t gets ``num_etype + t + 1`` (run_regnn.py:91-98).
    ``isolate`` nodes receive no in-edges except their self loop (deg == ew_self exercises clamp).
    """
    T = len(type_counts)
    N = int(sum(type_counts))
    ntype = np.repeat(np.arange(T), type_counts)
    allowed_dst = np.arange(isolate, N)
    src = rng.integers(0, N, size=n_edges)
    dst = rng.choice(allowed_dst, size=n_edges)
    keep = src != dst
    src, dst = src[keep], dst[keep]
    # duplicates (multigraph edges)
    di = rng.integers(0, src.size, size=n_dup)
    src = np.concatenate([src, src[di]])
    dst = np.concatenate([dst, dst[di]])
    pairs = ntype[src] * T + ntype[dst]
    uniq = np.unique(pairs)
    pair_id = {int(p): i + 1 for i, p in enumerate(uniq)}
    num_etype = len(uniq)
    rel = np.array([pair_id[int(p)] for p in pairs], dtype=np.int64)
    loops = np.arange(N)
    src = np.concatenate([src, loops]).astype(np.int64)
    dst = np.concatenate([dst, loops]).astype(np.int64)
    rel = np.concatenate([rel, num_etype + ntype + 1]).astype(np.int64)
    R = num_etype + T
    return dict(src=src, dst=dst, rel=rel, N=N, R=R, ntype=ntype.astype(np.int64),
                type_counts=np.asarray(type_counts, dtype=np.int64))


def f32(rng, *shape, scale=1.0):
    return (rng.standard_normal(shape) * scale).astype(np.float32)


def _set_params(module, rng, ew_alpha=None):
    """Overwrite every parameter with fp32-representable values (edge_weight: alpha*w in
    U(-0.5, 1.5) so both LeakyReLU slopes and the degree clamp are exercised)."""
    for name, p in module.named_parameters():
        leaf = name.split(".")[-1]
        if leaf in ("edge_weight", "relation_weight") and ew_alpha is not None:
            v = rng.uniform(-0.5, 1.5, size=tuple(p.shape)).astype(np.float32) / np.float32(ew_alpha)
            v = v.astype(np.float32)
        elif leaf == "bias" or "norm" in name or leaf.startswith("bn"):
            v = (rng.standard_normal(tuple(p.shape)) * 0.1).astype(np.float32)
            if "norm.weight" in name:
                v = (1.0 + v).astype(np.float32)
        else:
            v = f32(rng, *p.shape, scale=0.2)
        with torch.no_grad():
            p.copy_(torch.from_numpy(v.astype(np.float64)))


def _pack(prefix, d, store):
    for k, v in d.items():
        if isinstance(v, torch.Tensor):
            v = v.detach().cpu().numpy()
        v = np.asarray(v)
        if v.dtype == np.float64:
            v = v.astype(np.float32)
        store[prefix + k] = v


def _params(module):
    return {n: p.detach() for n, p in module.named_parameters()}


def _grads(module):
    return {n: p.grad for n, p in module.named_parameters() if p.grad is not None}


def save(name, meta, store):
    for k, v in list(store.items()):
        if isinstance(v, torch.Tensor):
            v = v.detach().cpu().numpy()
        if isinstance(v, np.ndarray) and v.dtype == np.float64:
            v = v.astype(np.float32)
        store[k] = v
    store["meta"] = np.array(json.dumps(meta))
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **store)
    print(f"wrote {path} ({os.path.getsize(path)//1024} KB)")


# ------------------------------------------------------------------------------------------
# full-batch layers (layer/*.py through the dgl shim)
# ------------------------------------------------------------------------------------------
def gen_layers():
    _purge(["dgl", "layer", "model", "utils"])
    _use_paths([SHIM, REF])
    import dgl
    layer = importlib.import_module("layer")
    import torch.nn.functional as F

    rng = np.random.default_rng(0)
    gd = make_hetero_graph(rng, [60, 70, 40, 30], 1800)
    g = dgl.DGLGraph((gd["src"], gd["dst"]), num_nodes=gd["N"])
    e_feat = torch.from_numpy(gd["rel"])
    N, R = gd["N"], gd["R"]

    # REGraphConv variants: (tag, in, out, kwargs)
    gcn_cases = [
        ("norm_noweight", 64, 64, dict(norm=True, bias=False, weight=False)),
        ("norm_weight_bias_elu", 64, 64, dict(norm=True, bias=True, weight=True, activation="elu")),
        ("nonorm_noweight", 64, 64, dict(norm=False, bias=False, weight=False)),
        ("norm_in_gt_out", 64, 32, dict(norm=True, bias=True, weight=True)),
        ("nonorm_in_lt_out", 32, 64, dict(norm=False, bias=True, weight=True)),
    ]
    alpha = 100.0
    for tag, fin, fout, kw in gcn_cases:
        kw = dict(kw)
        act = kw.pop("activation", None)
        torch.manual_seed(1)
        m = layer.REGraphConv(R, alpha, fin, fout, activation=F.elu if act else None, **kw)
        _set_params(m, rng, ew_alpha=alpha)
        feat = torch.from_numpy(f32(rng, N, fin).astype(np.float64)).requires_grad_(True)
        out = m(g, feat, e_feat)
        gout = f32(rng, *out.shape)
        out.backward(torch.from_numpy(gout.astype(np.float64)))
        st = {}
        _pack("g_", gd, st)
        st["feat"], st["gout"], st["out"] = feat.detach().numpy().astype(np.float32), gout, out
        st["grad_feat"] = feat.grad
        _pack("p_", _params(m), st)
        _pack("grad_", _grads(m), st)
        save(f"regraphconv_{tag}", dict(layer="REGraphConv", alpha=alpha, in_feats=fin,
                                         out_feats=fout, activation=act, **kw), st)

    # REGATConv variants
    gat_cases = [
        ("h4_ee", 32, 32, 4, dict(residual=False, use_weight=True), True, None),
        ("h4_noee", 32, 32, 4, dict(residual=False, use_weight=True), False, None),
        ("h8_d64_ee_res_elu", 48, 64, 8, dict(residual=True, use_weight=True), True, "elu"),
        ("h4_noweight_res", 128, 32, 4, dict(residual=True, use_weight=False), True, None),
    ]
    for tag, fin, fout, H, kw, use_ee, act in gat_cases:
        torch.manual_seed(2)
        m = layer.REGATConv(R, alpha, fin, fout, H, 0.0, 0.0, 0.01, kw["residual"],
                            F.elu if act else None, use_weight=kw["use_weight"])
        _set_params(m, rng, ew_alpha=alpha)
        feat = torch.from_numpy(f32(rng, N, fin).astype(np.float64)).requires_grad_(True)
        out = m(g, feat, e_feat if use_ee else None)
        gout = f32(rng, *out.shape)
        out.backward(torch.from_numpy(gout.astype(np.float64)))
        st = {}
        _pack("g_", gd, st)
        st["feat"], st["gout"], st["out"] = feat.detach().numpy().astype(np.float32), gout, out
        st["grad_feat"] = feat.grad
        _pack("p_", _params(m), st)
        _pack("grad_", _grads(m), st)
        save(f"regatconv_{tag}", dict(layer="REGATConv", alpha=alpha, in_feats=fin, out_feats=fout,
                                       num_heads=H, negative_slope=0.01, edge_feats=use_ee,
                                       activation=act, **kw), st)

    # REMixHopConv variants
    mix_cases = [("f64", 64, 64, None), ("f192_elu", 192, 64, "elu")]
    for tag, fin, fout, act in mix_cases:
        torch.manual_seed(3)
        m = layer.REMixHopConv(R, alpha, fin, fout, p=[0, 1, 2], dropout=0,
                               activation=F.elu if act else None, batchnorm=False)
        _set_params(m, rng, ew_alpha=alpha)
        feat = torch.from_numpy(f32(rng, N, fin).astype(np.float64)).requires_grad_(True)
        out = m(g, feat, e_feat)
        gout = f32(rng, *out.shape)
        out.backward(torch.from_numpy(gout.astype(np.float64)))
        st = {}
        _pack("g_", gd, st)
        st["feat"], st["gout"], st["out"] = feat.detach().numpy().astype(np.float32), gout, out
        st["grad_feat"] = feat.grad
        _pack("p_", _params(m), st)
        _pack("grad_", _grads(m), st)
        save(f"remixhopconv_{tag}", dict(layer="REMixHopConv", alpha=alpha, in_feats=fin,
                                          out_feats=fout, p=[0, 1, 2], activation=act), st)
    return gd


# ------------------------------------------------------------------------------------------
# whole models (model/*.py), eval mode / dropout 0
# ------------------------------------------------------------------------------------------
def gen_models():
    _purge(["dgl", "layer", "model", "utils"])
    _use_paths([SHIM, REF])
    import dgl
    import torch.nn.functional as F
    REGCN = importlib.import_module("model.REGCN").REGCN
    REGAT = importlib.import_module("model.REGAT").REGAT
    REMixHop = importlib.import_module("model.REMixHop").REMixHop

    rng = np.random.default_rng(10)
    type_counts = [50, 60, 30, 20]
    dims = [24, 40, 12, 20]
    gd = make_hetero_graph(rng, type_counts, 1500)
    g = dgl.DGLGraph((gd["src"], gd["dst"]), num_nodes=gd["N"])
    e_feat = torch.from_numpy(gd["rel"])
    R = gd["R"]
    alpha = 100.0
    n_classes = 4

    def run(tag, net, meta):
        _set_params(net, rng, ew_alpha=alpha)
        net.eval()
        feats = [torch.from_numpy(f32(rng, n, d).astype(np.float64))
                 for n, d in zip(type_counts, dims)]
        logits, emb = net(feats, e_feat)
        gout = f32(rng, *logits.shape)
        logits.backward(torch.from_numpy(gout.astype(np.float64)))
        st = {}
        _pack("g_", gd, st)
        for i, f in enumerate(feats):
            st[f"feat{i}"] = f.numpy().astype(np.float32)
        st["gout"], st["logits"], st["emb"] = gout, logits, emb
        _pack("p_", _params(net), st)
        _pack("grad_", _grads(net), st)
        meta.update(alpha=alpha, dims=dims, n_classes=n_classes)
        save(f"model_{tag}", meta, st)

    torch.manual_seed(4)
    run("regcn2", REGCN(g, R, alpha, 64, 64, n_classes, 2, F.elu, 0.0, dims),
        dict(model="REGCN", num_layers=2, hidden=64))
    torch.manual_seed(5)
    run("regcn4", REGCN(g, R, alpha, 64, 64, n_classes, 4, F.elu, 0.0, dims),
        dict(model="REGCN", num_layers=4, hidden=64))
    torch.manual_seed(6)
    heads = [8, 8, 1]
    run("regat2", REGAT(g, R, alpha, 2, 32, 32, n_classes, heads, F.elu, 0.0, 0.0, 0.01, False,
                        dims), dict(model="REGAT", num_layers=2, hidden=32, heads=heads))
    torch.manual_seed(7)
    run("remixhop2", REMixHop(g, R, alpha, 64, 64, n_classes, 2, dims, input_dropout=0.0,
                              activation=F.elu), dict(model="REMixHop", num_layers=2, hidden=64))


# ------------------------------------------------------------------------------------------
# mag REGCNConv (mag/regnn_layers.py) on a bipartite sampled block
# ------------------------------------------------------------------------------------------
def gen_mag():
    _purge(["dgl", "layer", "model", "utils", "regnn_layers", "torch_geometric", "torch_scatter",
            "torch_sparse", "ogb", "texttable"])
    _use_paths([SHIM, os.path.join(REF, "mag")])
    regnn_layers = importlib.import_module("regnn_layers")

    rng = np.random.default_rng(20)
    n_src, n_dst, E = 300, 100, 1500
    num_node_types, num_edge_types = 4, 7
    src = rng.integers(0, n_src, size=E).astype(np.int64)
    dst = rng.integers(0, n_dst, size=E).astype(np.int64)
    # a few targets with no sampled in-edges (only the appended self loop)
    dst[np.isin(dst, [3, 17, 42])] = 5
    edge_type = rng.integers(0, num_edge_types, size=E).astype(np.int64)
    tnt = rng.integers(0, num_node_types, size=n_dst).astype(np.int64)
    # (residual, use_softmax): the softmax case also records return_weights' ew (:119-121,137)
    for residual, use_softmax in ((False, False), (True, False), (False, True)):
        torch.manual_seed(8)
        conv = regnn_layers.REGCNConv(64, 64, num_node_types, num_edge_types, 10.0,
                                      use_softmax=use_softmax, residual=residual,
                                      use_norm="ln", self_loop_type=2)
        _set_params(conv, rng, ew_alpha=10.0)
        x = torch.from_numpy(f32(rng, n_src, 64).astype(np.float64)).requires_grad_(True)
        ei = torch.from_numpy(np.stack([src, dst]))
        res = conv((x, x[:n_dst]), ei, torch.from_numpy(edge_type), torch.from_numpy(tnt),
                   return_weights=use_softmax)
        out = res[0] if use_softmax else res
        gout = f32(rng, *out.shape)
        out.backward(torch.from_numpy(gout.astype(np.float64)))
        st = dict(src=src, dst=dst, edge_type=edge_type, target_node_type=tnt,
                  x=x.detach().numpy().astype(np.float32), gout=gout, out=out, grad_x=x.grad)
        if use_softmax:
            st["ew"] = res[1].detach()
        _pack("p_", _params(conv), st)
        _pack("grad_", _grads(conv), st)
        name = "mag_regcnconv_softmax" if use_softmax else f"mag_regcnconv_res{int(residual)}"
        save(name, dict(layer="mag.REGCNConv", n_src=n_src, n_dst=n_dst,
                        num_node_types=num_node_types, num_edge_types=num_edge_types,
                        scaling_factor=10.0, residual=residual, use_softmax=use_softmax,
                        use_norm="ln", self_loop_type=2), st)


# ------------------------------------------------------------------------------------------
# the other RE layers (layer/RESAGEConv.py, REGINConv.py, REGATv2Conv.py)
# ------------------------------------------------------------------------------------------
def gen_layers_extra():
    _purge(["dgl", "layer", "model", "utils"])
    _use_paths([SHIM, REF])
    import dgl
    layer = importlib.import_module("layer")
    import torch.nn.functional as F

    rng = np.random.default_rng(30)
    gd = make_hetero_graph(rng, [50, 60, 45, 25], 1600)
    g = dgl.DGLGraph((gd["src"], gd["dst"]), num_nodes=gd["N"])
    e_feat = torch.from_numpy(gd["rel"])
    N, R = gd["N"], gd["R"]
    alpha = 100.0

    def record(name, m, fin, meta, call):
        feat = torch.from_numpy(f32(rng, N, fin).astype(np.float64)).requires_grad_(True)
        out = call(m, feat)
        gout = f32(rng, *out.shape)
        out.backward(torch.from_numpy(gout.astype(np.float64)))
        st = {}
        _pack("g_", gd, st)
        st["feat"], st["gout"], st["out"] = feat.detach().numpy().astype(np.float32), gout, out
        st["grad_feat"] = feat.grad
        _pack("p_", _params(m), st)
        _pack("grad_", _grads(m), st)
        save(name, dict(alpha=alpha, in_feats=fin, **meta), st)

    sage_cases = [
        ("norm_weight_bias", 64, 64, dict(norm=True, bias=True, weight=True)),
        ("norm_in_gt_out_elu", 64, 32, dict(norm=True, bias=True, weight=True, activation="elu")),
        ("nonorm_noweight", 48, 48, dict(norm=False, bias=False, weight=False)),
    ]
    for tag, fin, fout, kw in sage_cases:
        kw = dict(kw)
        act = kw.pop("activation", None)
        torch.manual_seed(11)
        m = layer.RESAGEConv(R, alpha, fin, fout, activation=F.elu if act else None, **kw)
        _set_params(m, rng, ew_alpha=alpha)
        record(f"resageconv_{tag}", m, fin,
               dict(layer="RESAGEConv", out_feats=fout, activation=act, **kw),
               lambda m, f: m(g, f, e_feat))

    for tag, agg, lin in (("sum_linear", "sum", True), ("mean_nofunc", "mean", False)):
        torch.manual_seed(12)
        apply = torch.nn.Linear(64, 32) if lin else None
        m = layer.REGINConv(R, alpha, apply_func=apply, aggregator_type=agg)
        _set_params(m, rng, ew_alpha=alpha)
        record(f"reginconv_{tag}", m, 64, dict(layer="REGINConv", aggregator_type=agg,
                                               apply_linear=[64, 32] if lin else None),
               lambda m, f: m(g, f, e_feat))

    v2_cases = [
        ("h4_ee", 32, 16, 4, dict(residual=False, share_weights=False), True, None),
        ("h4_noee_share", 32, 16, 4, dict(residual=False, share_weights=True), False, None),
        ("h2_ee_res_elu", 24, 16, 2, dict(residual=True, share_weights=False), True, "elu"),
    ]
    for tag, fin, fout, H, kw, use_ee, act in v2_cases:
        torch.manual_seed(13)
        m = layer.REGATv2Conv(R, alpha, fin, fout, H, 0.0, 0.0, 0.2, kw["residual"],
                              F.elu if act else None, share_weights=kw["share_weights"])
        _set_params(m, rng, ew_alpha=alpha)
        record(f"regatv2conv_{tag}", m, fin,
               dict(layer="REGATv2Conv", out_feats=fout, num_heads=H, negative_slope=0.2,
                    edge_feats=use_ee, activation=act, **kw),
               lambda m, f: m(g, f, e_feat if use_ee else None))


def gen_mag_gat():
    """mag REGATConv / REGATv2Conv (mag/regnn_layers.py:153-436): global-max edge softmax."""
    _purge(["dgl", "layer", "model", "utils", "regnn_layers", "torch_geometric", "torch_scatter",
            "torch_sparse", "ogb", "texttable"])
    _use_paths([SHIM, os.path.join(REF, "mag")])
    regnn_layers = importlib.import_module("regnn_layers")
    rng = np.random.default_rng(40)
    n_src, n_dst, E = 260, 90, 1400
    num_node_types, num_edge_types = 4, 7
    src = rng.integers(0, n_src, size=E).astype(np.int64)
    dst = rng.integers(0, n_dst, size=E).astype(np.int64)
    dst[np.isin(dst, [2, 11])] = 4                  # targets with only their self loop
    edge_type = rng.integers(0, num_edge_types, size=E).astype(np.int64)
    tnt = rng.integers(0, num_node_types, size=n_dst).astype(np.int64)
    cases = [("regat", "REGATConv", 4, 16, False), ("regat", "REGATConv", 2, 32, True),
             ("regatv2", "REGATv2Conv", 4, 16, False), ("regatv2", "REGATv2Conv", 2, 32, True)]
    for tag, cls, H, C, residual in cases:
        torch.manual_seed(9)
        conv = getattr(regnn_layers, cls)(H * C, C, num_node_types, num_edge_types, heads=H,
                                          scaling_factor=10.0, residual=residual,
                                          use_norm="ln", self_loop_type=2)
        _set_params(conv, rng, ew_alpha=10.0)
        x = torch.from_numpy(f32(rng, n_src, H * C).astype(np.float64)).requires_grad_(True)
        ei = torch.from_numpy(np.stack([src, dst]))
        out = conv((x, x[:n_dst]), ei, torch.from_numpy(edge_type), torch.from_numpy(tnt))
        gout = f32(rng, *out.shape)
        out.backward(torch.from_numpy(gout.astype(np.float64)))
        st = dict(src=src, dst=dst, edge_type=edge_type, target_node_type=tnt,
                  x=x.detach().numpy().astype(np.float32), gout=gout, out=out, grad_x=x.grad)
        _pack("p_", _params(conv), st)
        _pack("grad_", _grads(conv), st)
        save(f"mag_{tag}conv_h{H}_res{int(residual)}",
             dict(layer=f"mag.{cls}", n_src=n_src, n_dst=n_dst, num_node_types=num_node_types,
                  num_edge_types=num_edge_types, heads=H, out_channels=C, scaling_factor=10.0,
                  residual=residual, use_norm="ln", self_loop_type=2, negative_slope=0.2), st)


# ------------------------------------------------------------------------------------------
# the REGNN model of mag/regnn_ns.py:216-346 (group_input feats_type 3 / 2, 2 x REGCNConv, relu,
# out_lin, log_softmax) + nll_loss (:404) on a sampled batch of a small typed graph
# ------------------------------------------------------------------------------------------
def _reference_regnn_class(args, num_nodes_dict, target_node_type, regnn_layers):
    """The reference's `class REGNN` is defined in the training script, whose top level parses
    argv and downloads ogbn-mag: compile ONLY that class definition (ast) against the globals it
    reads (args, num_nodes_dict, target_node_type, the layers)."""
    import ast
    from types import SimpleNamespace  # noqa: F401
    path = os.path.join(REF, "mag", "regnn_ns.py")
    tree = ast.parse(open(path).read(), path)
    cls = [n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == "REGNN"]
    assert len(cls) == 1
    code = compile(ast.Module(body=cls, type_ignores=[]), path, "exec")
    from torch.nn import Linear, ModuleDict, ModuleList, Parameter, ParameterDict
    ns = dict(torch=torch, F=torch.nn.functional, Linear=Linear, ModuleDict=ModuleDict,
              ModuleList=ModuleList, Parameter=Parameter, ParameterDict=ParameterDict,
              REGCNConv=regnn_layers.REGCNConv, REGATConv=regnn_layers.REGATConv,
              REGATv2Conv=regnn_layers.REGATv2Conv, args=args, num_nodes_dict=num_nodes_dict,
              target_node_type=target_node_type)
    exec(code, ns)
    return ns["REGNN"]


def gen_regnn():
    from types import SimpleNamespace
    _purge(["dgl", "layer", "model", "utils", "regnn_layers", "torch_geometric", "torch_scatter",
            "torch_sparse", "ogb", "texttable"])
    _use_paths([SHIM, os.path.join(REF, "mag")])
    regnn_layers = importlib.import_module("regnn_layers")
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    from oracle import sampler_oracle as SO
    rng = np.random.default_rng(50)
    counts = [40, 50, 8, 12]                       # paper (target), author, institution, field
    N = sum(counts)
    ntype = np.repeat(np.arange(4), counts)
    local = np.concatenate([np.arange(c) for c in counts])
    E = 900
    src = rng.integers(0, N, E)
    dst = rng.integers(0, N, E)
    dst[:40] = rng.integers(0, 3, 40)              # a few hub targets (rows longer than the fan-out)
    order = np.argsort(dst, kind="stable")         # edge ids = CSR positions of the dst-major CSR
    src, dst = src[order].astype(np.int64), dst[order].astype(np.int64)
    edge_type = rng.integers(0, 7, E).astype(np.int64)
    ptr = np.zeros(N + 1, np.int64)
    np.add.at(ptr, dst + 1, 1)
    ptr = np.cumsum(ptr)
    batch = rng.choice(counts[0], 12, replace=False).astype(np.int64)
    sizes, seed, epoch, batch_idx = [4, 3], 7, 1, 2
    _, n_id, adjs = SO.neighbor_sample(ptr, src, batch.tolist(), sizes, seed, epoch, batch_idx)
    K, H, C = 64, 64, 5
    y = rng.integers(0, C, counts[0]).astype(np.int64)
    for feats_type in (3, 2):
        args = SimpleNamespace(model="regcn", feats_type=feats_type, self_loop_type=2,
                               no_re=False)
        num_nodes_dict = {t: counts[t] for t in range(4)}
        REGNN = _reference_regnn_class(args, num_nodes_dict, 0, regnn_layers)
        torch.manual_seed(11)
        nfd = {t: K for t in range(4)}
        model = REGNN(K, H, C, 1, 2, 10.0, 0.0, nfd, 7, False, False, use_norm="ln")
        _set_params(model, rng, ew_alpha=10.0)
        model.eval()
        if feats_type == 3:
            x_dict = {t: torch.from_numpy(f32(rng, counts[t], K).astype(np.float64))
                      for t in range(4)}
        else:
            x_dict = {0: torch.from_numpy(f32(rng, counts[0], K).astype(np.float64))}
        t_adjs = [(torch.tensor([s_, d_], dtype=torch.int64), torch.tensor(e_, dtype=torch.int64),
                   sz) for s_, d_, e_, sz in adjs]
        out = model(torch.tensor(n_id), x_dict, t_adjs, torch.from_numpy(edge_type),
                    torch.from_numpy(ntype), torch.from_numpy(local))
        yb = torch.from_numpy(y[batch])
        loss = torch.nn.functional.nll_loss(out, yb)
        loss.backward()
        st = dict(src=src, dst=dst, edge_type=edge_type, ntype=ntype, local=local, y=y,
                  batch=batch, n_id=np.asarray(n_id, np.int64), logp=out, loss=loss.detach())
        for t, x in x_dict.items():
            st[f"x{t}"] = x.numpy().astype(np.float32)
        for h, (s_, d_, e_, sz) in enumerate(adjs):
            st[f"adj{h}_src"], st[f"adj{h}_dst"] = np.asarray(s_), np.asarray(d_)
            st[f"adj{h}_eid"] = np.asarray(e_)
            st[f"adj{h}_size"] = np.asarray(sz)
        _pack("p_", _params(model), st)
        _pack("grad_", _grads(model), st)
        save(f"mag_regnn_ft{feats_type}",
             dict(model="mag.REGNN", feats_type=feats_type, in_channels=K, hidden=H, classes=C,
                  num_layers=2, scaling_factor=10.0, num_edge_types=7, counts=counts,
                  sizes=sizes, seed=seed, epoch=epoch, batch_idx=batch_idx, use_norm="ln",
                  self_loop_type=2, dropout=0.0), st)


def _mag_schema_graph(rng, counts):
    """A small heterogeneous graph with ogbn-mag's schema, built the way mag/regnn_ns.py:91-105,
    141-142 builds the real one: the 4 raw relations (author-affiliated_with-institution,
    author-writes-paper, paper-cites-paper, paper-has_topic-field_of_study) in the dataset's
    edge_index_dict order, the 3 reverse relations appended, cites made undirected, then PyG's
    group_hetero_graph: node types numbered in num_nodes_dict order (ogbn-mag: author 0,
    field_of_study 1, institution 2, paper 3), global ids type by type, edge_type = the
    relation's position in edge_index_dict. [ext] PyG semantics restated here: to_undirected =
    coalesce(cat(ei, flip(ei))) (rows sorted by (row, col), duplicates dropped);
    group_hetero_graph concatenates the relations' edges in dict order. Every relation joins one
    source node type to one target node type (regnn_nsm_params.rel_slots holds)."""
    A, Fd, I, P = 0, 1, 2, 3
    off = np.concatenate([[0], np.cumsum(counts)[:-1]])

    def rnd(st, dt, n, hub_dst=None, hub_frac=0.0):
        s = rng.integers(0, counts[st], n)
        d = rng.integers(0, counts[dt], n)
        if hub_dst is not None:                       # a few hub targets: rows past the fan-out
            m = rng.random(n) < hub_frac
            d[m] = rng.integers(0, hub_dst, int(m.sum()))
        return np.stack([s, d])

    rels = {}
    rels[("author", "affiliated_with", "institution")] = (A, I, rnd(A, I, 260))
    rels[("author", "writes", "paper")] = (A, P, rnd(A, P, 700, hub_dst=3, hub_frac=0.12))
    cites = rnd(P, P, 500, hub_dst=2, hub_frac=0.1)
    rels[("paper", "has_topic", "field_of_study")] = (P, Fd, rnd(P, Fd, 420, hub_dst=2,
                                                                   hub_frac=0.15))
    r, c = rels[("author", "affiliated_with", "institution")][2]
    rels[("institution", "to", "author")] = (I, A, np.stack([c, r]))
    r, c = rels[("author", "writes", "paper")][2]
    rels[("paper", "to", "author")] = (P, A, np.stack([c, r]))
    r, c = rels[("paper", "has_topic", "field_of_study")][2]
    rels[("field_of_study", "to", "paper")] = (Fd, P, np.stack([c, r]))
    ei = np.concatenate([cites, cites[::-1]], 1)
    ei = np.unique(ei[0] * counts[P] + ei[1])
    cites = np.stack([ei // counts[P], ei % counts[P]])
    order = [("author", "affiliated_with", "institution"), ("author", "writes", "paper"),
             ("paper", "cites", "paper"), ("paper", "has_topic", "field_of_study"),
             ("institution", "to", "author"), ("paper", "to", "author"),
             ("field_of_study", "to", "paper")]
    rels[("paper", "cites", "paper")] = (P, P, cites)
    src, dst, et = [], [], []
    for i, key in enumerate(order):
        st, dt, e = rels[key]
        src.append(e[0] + off[st])
        dst.append(e[1] + off[dt])
        et.append(np.full(e.shape[1], i))
    src, dst, et = (np.concatenate(v).astype(np.int64) for v in (src, dst, et))
    o = np.argsort(dst, kind="stable")             # edge ids = CSR positions (dst-major, stable)
    ntype = np.repeat(np.arange(4), counts).astype(np.int64)
    local = np.concatenate([np.arange(c) for c in counts]).astype(np.int64)
    return src[o], dst[o], et[o], ntype, local, int(off[P])


def gen_regnn_schema():
    """The benchmarked NS mode pinned to the reference: the reference REGNN
    on an ogbn-mag-schema graph (one relation per (source type, target type) pair: the fused
    step's relation-slot mode applies), K = 128 input rows (feats_type 3), hidden 64, 349
    classes, fan-out [25, 20] (mag/regnn_ns.py defaults), dropout 0, nll_loss, every gradient."""
    from types import SimpleNamespace
    _purge(["dgl", "layer", "model", "utils", "regnn_layers", "torch_geometric", "torch_scatter",
            "torch_sparse", "ogb", "texttable"])
    _use_paths([SHIM, os.path.join(REF, "mag")])
    regnn_layers = importlib.import_module("regnn_layers")
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    from oracle import sampler_oracle as SO
    rng = np.random.default_rng(77)
    counts = [170, 40, 14, 130]                    # author, field_of_study, institution, paper
    src, dst, edge_type, ntype, local, p0 = _mag_schema_graph(rng, counts)
    N = int(sum(counts))
    ptr = np.zeros(N + 1, np.int64)
    np.add.at(ptr, dst + 1, 1)
    ptr = np.cumsum(ptr)
    batch = (p0 + rng.choice(counts[3], 24, replace=False)).astype(np.int64)
    batch[:3] = p0 + np.arange(3)                  # the hub papers among the targets
    sizes, seed, epoch, batch_idx = [25, 20], 123, 0, 5
    _, n_id, adjs = SO.neighbor_sample(ptr, src, batch.tolist(), sizes, seed, epoch, batch_idx)
    K, H, C = 128, 64, 349
    y = np.full(N, -1, np.int64)
    y[p0:] = rng.integers(0, C, counts[3])
    args = SimpleNamespace(model="regcn", feats_type=3, self_loop_type=2, no_re=False)
    REGNN = _reference_regnn_class(args, {t: counts[t] for t in range(4)}, 3, regnn_layers)
    torch.manual_seed(12)
    model = REGNN(K, H, C, 1, 2, 10.0, 0.0, {t: K for t in range(4)}, 7, False, False,
                  use_norm="ln")
    _set_params(model, rng, ew_alpha=10.0)
    model.eval()
    x_dict = {t: torch.from_numpy((f32(rng, counts[t], K) if t == 3 else
                                   rng.uniform(-0.5, 0.5, (counts[t], K)).astype(np.float32))
                                  .astype(np.float64)) for t in range(4)}
    t_adjs = [(torch.tensor([s_, d_], dtype=torch.int64), torch.tensor(e_, dtype=torch.int64), sz)
              for s_, d_, e_, sz in adjs]
    out = model(torch.tensor(n_id), x_dict, t_adjs, torch.from_numpy(edge_type),
                torch.from_numpy(ntype), torch.from_numpy(local))
    loss = torch.nn.functional.nll_loss(out, torch.from_numpy(y[batch]))
    loss.backward()
    st = dict(src=src, dst=dst, edge_type=edge_type, ntype=ntype, local=local, y=y, batch=batch,
              n_id=np.asarray(n_id, np.int64), logp=out, loss=loss.detach())
    for t, x in x_dict.items():
        st[f"x{t}"] = x.numpy().astype(np.float32)
    for h, (s_, d_, e_, sz) in enumerate(adjs):
        st[f"adj{h}_src"], st[f"adj{h}_dst"] = np.asarray(s_), np.asarray(d_)
        st[f"adj{h}_eid"] = np.asarray(e_)
        st[f"adj{h}_size"] = np.asarray(sz)
    _pack("p_", _params(model), st)
    _pack("grad_", _grads(model), st)
    save("mag_regnn_schema", dict(model="mag.REGNN", feats_type=3, in_channels=K, hidden=H,
                                  classes=C, num_layers=2, scaling_factor=10.0, num_edge_types=7,
                                  counts=counts, target_type=3, target_offset=p0, y_global=True,
                                  sizes=sizes, seed=seed, epoch=epoch, batch_idx=batch_idx,
                                  use_norm="ln", self_loop_type=2, dropout=0.0,
                                  schema="ogbn-mag"), st)


def gen_regnn_ft5():
    """The reference's default NS model shape: the reference REGNN on the
    ogbn-mag-schema graph with feats_type 5's unequal input widths (mag/regnn_ns.py:185-194:
    paper rows = cat(raw 128-d, a 128-d embedding) = 256-d, every other type a 128-d embedding),
    hidden 128, residual on (:62), LayerNorm, 349 classes, fan-out [25, 20], dropout 0: loss and
    every gradient."""
    from types import SimpleNamespace
    _purge(["dgl", "layer", "model", "utils", "regnn_layers", "torch_geometric", "torch_scatter",
            "torch_sparse", "ogb", "texttable"])
    _use_paths([SHIM, os.path.join(REF, "mag")])
    regnn_layers = importlib.import_module("regnn_layers")
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    from oracle import sampler_oracle as SO
    rng = np.random.default_rng(91)
    counts = [150, 36, 12, 120]                    # author, field_of_study, institution, paper
    src, dst, edge_type, ntype, local, p0 = _mag_schema_graph(rng, counts)
    N = int(sum(counts))
    ptr = np.zeros(N + 1, np.int64)
    np.add.at(ptr, dst + 1, 1)
    ptr = np.cumsum(ptr)
    batch = (p0 + rng.choice(counts[3], 20, replace=False)).astype(np.int64)
    batch[:2] = p0 + np.arange(2)
    sizes, seed, epoch, batch_idx = [25, 20], 5, 2, 3
    _, n_id, adjs = SO.neighbor_sample(ptr, src, batch.tolist(), sizes, seed, epoch, batch_idx)
    H, C = 128, 349
    dims = {0: 128, 1: 128, 2: 128, 3: 256}
    y = np.full(N, -1, np.int64)
    y[p0:] = rng.integers(0, C, counts[3])
    args = SimpleNamespace(model="regcn", feats_type=5, self_loop_type=2, no_re=False)
    REGNN = _reference_regnn_class(args, {t: counts[t] for t in range(4)}, 3, regnn_layers)
    torch.manual_seed(13)
    model = REGNN(128, H, C, 1, 2, 10.0, 0.0, dims, 7, True, False, use_norm="ln")
    _set_params(model, rng, ew_alpha=10.0)
    model.eval()
    x_dict = {t: torch.from_numpy(f32(rng, counts[t], dims[t], scale=0.5).astype(np.float64))
              for t in range(4)}
    t_adjs = [(torch.tensor([s_, d_], dtype=torch.int64), torch.tensor(e_, dtype=torch.int64), sz)
              for s_, d_, e_, sz in adjs]
    out = model(torch.tensor(n_id), x_dict, t_adjs, torch.from_numpy(edge_type),
                torch.from_numpy(ntype), torch.from_numpy(local))
    loss = torch.nn.functional.nll_loss(out, torch.from_numpy(y[batch]))
    loss.backward()
    st = dict(src=src, dst=dst, edge_type=edge_type, ntype=ntype, local=local, y=y, batch=batch,
              n_id=np.asarray(n_id, np.int64), logp=out, loss=loss.detach())
    for t, x in x_dict.items():
        st[f"x{t}"] = x.numpy().astype(np.float32)
    for h, (s_, d_, e_, sz) in enumerate(adjs):
        st[f"adj{h}_src"], st[f"adj{h}_dst"] = np.asarray(s_), np.asarray(d_)
        st[f"adj{h}_eid"] = np.asarray(e_)
        st[f"adj{h}_size"] = np.asarray(sz)
    _pack("p_", _params(model), st)
    _pack("grad_", _grads(model), st)
    save("mag_regnn_ft5_h128", dict(model="mag.REGNN", feats_type=5, in_channels=128, hidden=H,
                                    classes=C, num_layers=2, scaling_factor=10.0,
                                    num_edge_types=7, counts=counts, target_type=3,
                                    target_offset=p0, y_global=True, sizes=sizes, seed=seed,
                                    epoch=epoch, batch_idx=batch_idx, use_norm="ln",
                                    self_loop_type=2, dropout=0.0, schema="ogbn-mag",
                                    residual=True, feature_dims=[dims[t] for t in range(4)]), st)


def gen_regnn_init():
    """Seeded initial parameters of the reference's REGNN (mag/regnn_ns.py:216-298: every module
    constructed, then reset_parameters() again; REGCNConv draws weight_root = weight a second
    time when residual, mag/regnn_layers.py:71-78) for a few configurations, drawn in float32
    (the dtype the build's modules are created in): the build must consume the same RNG stream."""
    from types import SimpleNamespace
    _purge(["dgl", "layer", "model", "utils", "regnn_layers", "torch_geometric", "torch_scatter",
            "torch_sparse", "ogb", "texttable"])
    _use_paths([SHIM, os.path.join(REF, "mag")])
    regnn_layers = importlib.import_module("regnn_layers")
    prev = torch.get_default_dtype()
    torch.set_default_dtype(torch.float32)
    cfgs = [dict(feats_type=3, hidden=64, residual=False, dims=[128, 128, 128, 128], seed=3),
            dict(feats_type=5, hidden=128, residual=True, dims=[128, 128, 128, 256], seed=4),
            dict(feats_type=2, hidden=64, residual=True, dims=[128, 128, 128, 128], seed=6)]
    counts = {0: 30, 1: 9, 2: 5, 3: 20}
    st, meta = {}, []
    try:
        for i, c in enumerate(cfgs):
            args = SimpleNamespace(model="regcn", feats_type=c["feats_type"], self_loop_type=2,
                                   no_re=False)
            REGNN = _reference_regnn_class(args, counts, 3, regnn_layers)
            torch.manual_seed(c["seed"])
            m = REGNN(128, c["hidden"], 349, 1, 2, 10.0, 0.5,
                      {t: c["dims"][t] for t in range(4)}, 7, c["residual"], False,
                      use_norm="ln")
            _pack(f"c{i}_p_", _params(m), st)
            meta.append(dict(c, counts=[counts[t] for t in range(4)], target_type=3,
                             classes=349, num_layers=2, scaling_factor=10.0, dropout=0.5,
                             num_edge_types=7, in_channels=128))
    finally:
        torch.set_default_dtype(prev)
    save("mag_regnn_init", dict(configs=meta), st)


if __name__ == "__main__":
    torch.set_default_dtype(torch.float64)
    which = sys.argv[1:] or ["layers", "models", "mag", "extra", "maggat", "regnn", "schema",
                             "ft5", "init"]
    if "layers" in which:
        gen_layers()
    if "models" in which:
        gen_models()
    if "mag" in which:
        gen_mag()
    if "extra" in which:
        gen_layers_extra()
    if "maggat" in which:
        gen_mag_gat()
    if "regnn" in which:
        gen_regnn()
    if "schema" in which:
        gen_regnn_schema()
    if "ft5" in which:
        gen_regnn_ft5()
    if "init" in which:
        gen_regnn_init()
