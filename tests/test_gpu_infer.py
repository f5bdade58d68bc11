"""GPU parity of the layer-wise full-neighbour inference (mag/regnn_ns.py:348-369) against the
fp64 oracle (oracle.regnn_oracle.MagREGCNConvOracle over the full graph with every in-edge), on
one rank and with the rows sharded over 3 ranks driven in lockstep inside one process (the
exchange is then a concatenation; tests/test_cpu_infer.py covers the gloo all-gather)."""
import numpy as np
import pytest
import torch

import _golden as G
from oracle import regnn_oracle as O
from test_gpu_ns import _setup

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _oracle_inference(gd, rg, edge_type, node_type, local, x_dict, model):
    P = {n: p.detach().double().cpu().numpy() for n, p in model.named_parameters()}
    nt = node_type.cpu().numpy()
    loc = local.cpu().numpy()
    N = nt.size
    x = np.zeros((N, model.hidden_dim))
    for k, xf in x_dict.items():
        m = nt == k
        x[m] = xf.double().cpu().numpy()[loc[m]] @ P[f"lins.{k}.weight"].T + P[f"lins.{k}.bias"]
    eid = rg.csr_eid.cpu().numpy()
    src = rg.csr_idx.cpu().numpy().astype(np.int64)
    dst = np.repeat(np.arange(N), np.diff(rg.csr_ptr.cpu().numpy()))
    et = edge_type.cpu().numpy()[eid]
    for i in range(model.num_layers):
        pc = {k[len(f"convs.{i}."):]: v for k, v in P.items() if k.startswith(f"convs.{i}.")}
        o = O.MagREGCNConvOracle(N, 7, 10.0, residual=model.convs[i].residual, use_norm="ln")
        x = np.maximum(o.forward(x, src, dst, et, nt, pc), 0)
    return x @ P["out_lin.weight"].T + P["out_lin.bias"]


@pytest.mark.parametrize("residual", [False, True])
def test_full_neighbour_inference(residual):
    from regnn_hip import mag
    from regnn_hip.sampler import NeighborSampler
    gd, rg, edge_type, node_type, local, x_dict, model = _setup(scale=0.002)
    if residual:
        for c in model.convs:
            c.residual = True
    model.eval()
    loader = NeighborSampler(rg, None, [-1], batch_size=4096, shuffle=False)
    out = model.inference(x_dict, loader, edge_type, node_type, local, DEV)
    ref = _oracle_inference(gd, rg, edge_type, node_type, local, x_dict, model)
    assert out.shape == ref.shape
    ok, err = G.close(out.cpu().numpy(), ref, 1e-5)
    assert ok, f"inference rel err {err:.3e}"


def test_sharded_inference_lockstep():
    from regnn_hip.inference import ShardedInference, shard_bounds
    gd, rg, edge_type, node_type, local, x_dict, model = _setup(scale=0.002, seed=2)
    model.eval()
    W = 3
    bounds = shard_bounds(rg.csr_ptr, W)
    ranks = [ShardedInference(model, rg, edge_type, node_type, local, r, W, bounds)
             for r in range(W)]
    xs = [s.input(x_dict, 0)[1] for s in ranks]
    for layer in range(model.num_layers):
        xs_all = torch.cat(xs, 0)                        # what exchange_rows returns
        xl = [s.aggregate(layer, xs_all, xr) for s, xr in zip(ranks, xs)]
        if layer + 1 < model.num_layers:
            xs = [s.project(layer + 1, x) for s, x in zip(ranks, xl)]
    out = torch.cat([s.head(x) for s, x in zip(ranks, xl)], 0)
    ref = _oracle_inference(gd, rg, edge_type, node_type, local, x_dict, model)
    ok, err = G.close(out.cpu().numpy(), ref, 1e-5)
    assert ok, f"sharded inference rel err {err:.3e}"
    one = ShardedInference(model, rg, edge_type, node_type, local).run(x_dict)
    assert torch.allclose(out, one, rtol=1e-5, atol=1e-5)


def test_inference_argmax_head():
    """gather='argmax' runs the MFMA head without logits (regnn_head_argmax): equals the argmax
    of the oracle logits wherever the top two classes are not within fp32 noise."""
    from regnn_hip.inference import ShardedInference
    gd, rg, edge_type, node_type, local, x_dict, model = _setup(scale=0.002, seed=4)
    model.eval()
    am = ShardedInference(model, rg, edge_type, node_type, local).run(x_dict, gather="argmax")
    ref = _oracle_inference(gd, rg, edge_type, node_type, local, x_dict, model)
    top2 = np.sort(ref, 1)[:, -2:]
    clear = (top2[:, 1] - top2[:, 0]) > 1e-4
    got = am.cpu().numpy()
    assert am.dtype == torch.int64 and got.shape == (ref.shape[0],)
    assert np.array_equal(got[clear], ref.argmax(1)[clear])
    assert clear.mean() > 0.9


def test_head_argmax_ties_and_widths():
    from regnn_hip import ops
    g = torch.Generator().manual_seed(0)
    for C in (5, 16, 37, 349):
        h = torch.randn(1000, 64, generator=g).to(DEV)
        W = torch.randn(C, 64, generator=g).to(DEV)
        b = torch.randn(C, generator=g).to(DEV)
        z = torch.addmm(b, h, W.t())
        got = ops.head_argmax(h, W, b)
        top2 = torch.topk(z, min(2, C), 1).values
        clear = (top2[:, 0] - top2[:, -1]) > 1e-4 if C > 1 else torch.ones(1000, dtype=torch.bool)
        assert torch.equal(got[clear], z.argmax(1)[clear])
    W = torch.zeros(20, 64, device=DEV)                      # all classes tie -> class 0
    assert int(ops.head_argmax(torch.randn(64, 64, device=DEV), W).max()) == 0
