"""Benchmark: REGCN (2 x REGraphConv, hidden 64) full training step on a synthetic
ogbn-mag-scale multi-relation graph — BASELINE.json metric "aggregated edges/sec per GPU
(REGCN fwd+bwd, hidden=64); % HBM roofline".

One step = per-type input Linear -> REGraphConv x2 (HIP degree + SpMM) -> out_lin -> CE loss ->
backward (HIP fused transposed SpMM + SDDMM + relation/degree grads) -> Adam. Inputs resident in
HBM before timing. value = n_gpus * L * E / t_step (aggregated edges/s, whole job).

Multi-GPU: the full-batch path does not shard -> every rank trains an
independent replica on its own copy of the graph ("replicas only", weak scaling, no collective
in the timed region). Launch: python -m torch.distributed.run --nproc-per-node N bench.py --gpus N

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload mag|dblp] [--scale 10]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "re-gnn_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import torch.nn.functional as F  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X spec (MI355X_MICROARCH.md: 8.0 TB/s)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def setup_dist(n):
    if n > 1 or int(os.environ.get("WORLD_SIZE", "1")) > 1:
        dist.init_process_group("nccl")
        rank, world = dist.get_rank(), dist.get_world_size()
        local = int(os.environ.get("LOCAL_RANK", rank))
    else:
        rank, world, local = 0, 1, 0
    torch.cuda.set_device(local)
    return rank, world, torch.device("cuda", local)


def build_workload(args, dev):
    import dgl
    from regnn_hip import nets, synth
    t0 = time.time()
    if args.workload == "mag":
        gd = synth.mag_like(args.scale, seed=0, device=dev)
        dims = {t: 128 for t in synth.NTYPES}
        feats = synth.type_features(gd["counts"], dims, seed=1, device=dev, kind="mag")
        n_classes = 349
        train_nodes = gd["counts"]["paper"]
    else:
        gd = synth.dblp_like(seed=0, device=dev)
        feats = synth.type_features(gd["counts"], synth.DBLP_DIMS, seed=1, device=dev, kind="dblp")
        n_classes = 4
        train_nodes = gd["counts"]["A"]
    g = dgl.DGLGraph((gd["src"], gd["dst"]), num_nodes=gd["N"])
    e_feat = gd["rel"].to(torch.int64)
    rg = g.relgraph(dev)
    gen = torch.Generator(device=dev)
    gen.manual_seed(2)
    labels = torch.randint(0, n_classes, (train_nodes,), generator=gen, device=dev)
    torch.manual_seed(3)
    net = nets.REGCN(g, gd["R"], 100.0, 64, 64, n_classes, 2, F.elu, args.dropout,
                     [f.shape[1] for f in feats]).to(dev)
    opt = torch.optim.Adam(net.parameters(), lr=1e-3, weight_decay=1e-3)
    torch.cuda.synchronize()
    log(f"[bench] {args.workload}: N={gd['N']:,} E={rg.E:,} R={gd['R']} built in "
        f"{time.time() - t0:.1f}s; long rows csr={rg.csr_plan.n_long} csc={rg.csc_plan.n_long}")
    return dict(g=g, rg=rg, net=net, opt=opt, feats=feats, e_feat=e_feat, labels=labels, gd=gd)


def train_step(w):
    net, opt = w["net"], w["opt"]
    logits, _ = net(w["feats"], w["e_feat"])
    # = F.cross_entropy(logits[train], y) (run_regnn.py:147); gather form: torch's nll_loss
    # reduction is a single-block kernel (17 ms at 7.4M rows, profiled)
    logp = F.log_softmax(logits[: w["labels"].numel()], dim=1)
    loss = -logp.gather(1, w["labels"].unsqueeze(1)).mean()
    opt.zero_grad(set_to_none=True)
    loss.backward()
    opt.step()
    return loss


def spmm_bytes(E, N, F, s, kind):
    """algorithmic HBM bytes of one launch: int32 idx, uint8 rel, fp32 norm."""
    if kind == "spmm_fwd":      # gather row + idx 4 + rel 1 + norm[src] 4; ptr 8, norm 4, out row
        return E * (F * s + 9) + N * (F * s + 8)
    if kind == "spmm_bwd":      # gather g row + idx + rel + norm; per node x, g, out rows + misc
        return E * (F * s + 9) + N * (3 * F * s + 12)
    raise KeyError(kind)


def cpu_baseline(budget_s=20.0):
    """oracle ("port": numpy/scipy restatement) REGCN-2 fwd+bwd, hidden 64, on a bounded
    mag-shaped sample, single thread; returns (edges/s, sample description)."""
    import scipy.sparse  # noqa: F401
    from oracle import regnn_oracle as O
    from regnn_hip import synth
    scale = 0.01
    gd = synth.mag_like(scale, seed=0, device="cpu")
    src, dst = gd["src"].numpy(), gd["dst"].numpy()
    rel = gd["rel"].numpy().astype(np.int64)
    N, E = gd["N"], src.size
    g = O.Graph(src, dst, N)
    rng = np.random.default_rng(0)
    h = rng.standard_normal((N, 64)).astype(np.float32)
    ew = np.full((gd["R"], 1), 0.01, dtype=np.float32)
    layers = [O.REGraphConvOracle(100.0, 64, 64) for _ in range(2)]
    t0 = time.perf_counter()
    steps = 0
    while True:
        x = h
        for lay in layers:
            x = lay.forward(g, x, rel, ew)
        gx = x.copy()
        for lay in reversed(layers):
            gx, _ = lay.backward(g, gx)
        steps += 1
        el = time.perf_counter() - t0
        if el > budget_s or steps >= 50:
            break
    return 2 * E * steps / el, f"mag_like(scale={scale}) N={N:,} E={E:,}, {steps} fwd+bwd steps"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=["mag", "dblp"], default="mag")
    ap.add_argument("--scale", type=float, default=10.0)
    ap.add_argument("--dropout", type=float, default=0.5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    rank, world, dev = setup_dist(args.gpus)
    from regnn_hip import profile

    w = build_workload(args, dev)
    rg = w["rg"]
    for _ in range(args.warmup):
        train_step(w)
    torch.cuda.synchronize()

    profile.enable(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        train_step(w)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kstats = profile.summary()
    profile.enable(False)
    if world > 1:
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    ms = elapsed / args.steps * 1e3
    L = 2
    value = world * L * rg.E / (ms / 1e3)

    # dominant HIP kernel and its roofline
    F_, s = 64, 4
    cand = {k: v for k, v in kstats.items() if k in ("spmm_fwd", "spmm_bwd")}
    dom = max(cand, key=lambda k: cand[k][2])
    launches, mean_ms, _ = cand[dom]
    byts = spmm_bytes(rg.E, rg.n_dst, F_, s, dom)
    achieved = byts / (mean_ms / 1e3) / 1e9
    # HBM traffic per launch from the committed rocprofv3 PMC passes (tools/gpu_pmc.sh:
    # FETCH_SIZE and WRITE_SIZE in separate runs, calibrated on a 4 GiB copy), valid only for the
    # exact graph it was measured on
    traffic = None
    pmc = os.path.join(ROOT, "profiles", f"pmc_{args.workload}.json")
    if os.path.exists(pmc):
        with open(pmc) as f:
            rec = json.load(f)
        if rec.get("graph") == {"N": rg.n_dst, "E": rg.E} and dom in rec:
            traffic = rec[dom]["bytes_per_launch"]

    result = {
        "metric": "aggregated edges/sec per GPU (REGCN fwd+bwd, hidden=64); % HBM roofline",
        "value": value,
        "unit": "edges/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic (seeded ogbn-mag-shaped multi-relation graph, random features/labels)",
        "config": {
            "workload": (f"REGCN 2-layer hidden=64 full-graph train step (input Linear, "
                         f"2x REGraphConv fwd+bwd, out_lin, CE, Adam) on mag_like(scale="
                         f"{args.scale})" if args.workload == "mag" else
                         "REGCN 2-layer hidden=64 full-graph train step on dblp_like"),
            "nodes": rg.n_dst, "edges": rg.E, "relations": w["gd"]["R"], "layers": L,
            "hidden": 64, "parallelism": f"replicas x{world}",
        },
        "roofline": {
            "bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
            "launch_ms": mean_ms, "launches": launches, "algorithmic_bytes_per_launch": byts,
        },
        "kernels_ms": {k: round(v[1], 4) for k, v in kstats.items()},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        v, desc = cpu_baseline()
        result["cpu_baseline"] = {"value": v, "unit": "edges/s", "cores": 1, "kind": "port",
                                  "sample": desc + " (oracle/regnn_oracle.py numpy/scipy fp32)"}
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
