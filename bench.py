"""Benchmark: REGCN (2 x REGraphConv, hidden 64) full training step on a synthetic
ogbn-mag-scale multi-relation graph — BASELINE.json metric "aggregated edges/sec per GPU
(REGCN fwd+bwd, hidden=64); % HBM roofline".

One step = per-type input Linear -> REGraphConv x2 (HIP degree + SpMM) -> out_lin -> CE loss ->
backward (HIP fused transposed SpMM + SDDMM + relation/degree grads) -> Adam. Inputs resident in
HBM before timing. value = n_gpus * L * E / t_step (aggregated edges/s, whole job).

Multi-GPU (full-batch workloads): graph-shard data parallelism, weak scaling. Every rank holds
its own graph shard of the configured size (the same generator, seeded by rank: rank 0's shard is
the N=1 graph) and the same replicated parameters; after backward one flat-bucket RCCL
all-reduce averages the gradients (mag.flat_grad_allreduce, the DP exchange of
mag/regnn_ns.py:406-407) and every rank applies the same Adam step, so the ranks train one model.
The shards have no cross-shard edges (a whole graph fits one GPU: SURVEY.md §8e), so there is no
halo exchange. The neighbour-sampled path (--workload ns) is the reference's own DP path.
Launch: python -m torch.distributed.run --nproc-per-node N bench.py --gpus N

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
        # RCCL ("nccl"); REGNN_DIST_BACKEND=gloo rehearses several ranks on one device
        dist.init_process_group(os.environ.get("REGNN_DIST_BACKEND", "nccl"))
        rank, world = dist.get_rank(), dist.get_world_size()
        local = int(os.environ.get("LOCAL_RANK", rank))
    else:
        rank, world, local = 0, 1, 0
    local %= max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    return rank, world, torch.device("cuda", local)


def _full_graph(gd, dev):
    import dgl
    g = dgl.DGLGraph((gd["src"], gd["dst"]), num_nodes=gd["N"])
    return g, g.relgraph(dev), gd["rel"].to(torch.int64)


def build_workload(args, dev):
    """-> dict(step=callable, edges_per_step=int|callable, rg=RelGraph, kernels=[...], ...)."""
    from regnn_hip import mag, nets, ops, synth
    t0 = time.time()
    wl = args.workload
    rank = dist.get_rank() if dist.is_initialized() else 0
    world = dist.get_world_size() if dist.is_initialized() else 1
    gen = torch.Generator(device=dev)
    gen.manual_seed(2 + 1000 * rank)
    torch.manual_seed(3)              # identical parameter init on every rank
    gs, fs = rank, 1 + 1000 * rank    # graph / feature seeds of this rank's shard
    if wl in ("mag", "dblp"):
        if wl == "mag":
            gd = synth.mag_like(args.scale, seed=gs, device=dev)
            feats = synth.type_features(gd["counts"], {t: 128 for t in synth.NTYPES}, seed=fs,
                                        device=dev, kind="mag")
            n_classes, train_nodes = 349, gd["counts"]["paper"]
        else:
            gd = synth.dblp_like(seed=gs, device=dev)
            feats = synth.type_features(gd["counts"], synth.DBLP_DIMS, seed=fs, device=dev,
                                        kind="dblp")
            n_classes, train_nodes = 4, gd["counts"]["A"]
        g, rg, e_feat = _full_graph(gd, dev)
        net = nets.REGCN(g, gd["R"], 100.0, 64, 64, n_classes, 2, F.elu, args.dropout,
                         [f.shape[1] for f in feats]).to(dev)
        if args.dtype == "bf16":
            # BASELINE configs[1]: bf16 feature storage (input features, hidden rows), fp32 master
            # weights, fp32 accumulation in every kernel
            feats = [f.to(torch.bfloat16) for f in feats]
        convs, kern = 2, ("spmm_fwd", "spmm_bwd")
    elif wl == "acm":
        gd = synth.acm_like(seed=gs, device=dev)
        feats = synth.type_features(gd["counts"], synth.ACM_DIMS, seed=fs, device=dev, kind="target")
        n_classes, train_nodes = 3, gd["counts"]["P"]
        g, rg, e_feat = _full_graph(gd, dev)
        net = nets.REGAT(g, gd["R"], 100.0, 2, 64, 64, n_classes, [8, 8, 1], F.elu, args.dropout,
                         args.dropout, 0.01, False, [f.shape[1] for f in feats]).to(dev)
        convs, kern = 3, ("spmm_heads_fwd", "spmm_heads_bwd", "gat_softmax_fwd", "gat_softmax_bwd")
    elif wl == "imdb":
        gd = synth.imdb_like(seed=gs, device=dev)
        feats = synth.type_features(gd["counts"], synth.IMDB_DIMS, seed=fs, device=dev, kind="target")
        n_classes, train_nodes = 3, gd["counts"]["M"]
        g, rg, e_feat = _full_graph(gd, dev)
        net = nets.REMixHop(g, gd["R"], 100.0, 64, 64, n_classes, 2, [f.shape[1] for f in feats],
                            input_dropout=args.dropout, activation=F.elu).to(dev)
        convs, kern = 4, ("spmm_fwd", "spmm_bwd")        # 2 live hops x 2 layers
    elif wl == "ns_infer":
        return build_ns_infer(args, dev, t0)
    else:
        return build_ns(args, dev, t0)
    labels = torch.randint(0, n_classes, (train_nodes,), generator=gen, device=dev)
    # capturable: Adam's step counters live on the device so the step can be HIP-graph captured
    opt = torch.optim.Adam(net.parameters(), lr=1e-3, weight_decay=1e-3, capturable=True)

    W, b = net.head()
    params = list(net.parameters())

    def step():
        # run_regnn.py:146-150: logits = net(...) over all nodes, CE on the train rows, backward,
        # Adam. ops.head_ce computes the same logits / loss / gradients without the all-rows
        # zero-filled logits gradient (tests/test_gpu_ops.py::test_head_ce checks it vs autograd)
        _, loss = ops.head_ce(net.embed(feats, e_feat), W, b, labels)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        if world > 1:
            mag.flat_grad_allreduce(params, world)      # DP exchange (RCCL over xGMI)
        opt.step()

    torch.cuda.synchronize()
    log(f"[bench] {wl}: N={gd['N']:,} E={rg.E:,} R={gd['R']} built in {time.time() - t0:.1f}s; "
        f"long rows csr={rg.csr_plan.n_long} csc={rg.csc_plan.n_long}")
    return dict(step=step, edges_per_step=convs * rg.E, rg=rg, R=gd["R"], kernels=kern,
                convs=convs, N=rg.n_dst, E=rg.E, opt=opt)


def build_ns(args, dev, t0):
    """config 5: mag/regnn_ns.py REGCN neighbour-sampled training step (sample + fwd/bwd + Adam),
    data-parallel over ranks with the flat-bucket gradient all-reduce."""
    from regnn_hip import mag, synth
    from regnn_hip.graph import RelGraph
    from regnn_hip.sampler import NeighborSampler
    gd = synth.mag_like(args.scale, seed=0, device=dev)
    keep = gd["rel"] <= 7                                  # the raw 7 edge types, no loops
    src, dst = gd["src"][keep], gd["dst"][keep]
    edge_type = (gd["rel"][keep].to(torch.int64) - 1)
    rg = RelGraph(src, dst, gd["N"], dev)
    node_type = gd["ntype"]
    offs = torch.tensor([gd["type_offsets"][t] for t in synth.NTYPES], device=dev)
    local_node_idx = torch.arange(gd["N"], device=dev) - offs[node_type]
    feats = synth.type_features(gd["counts"], {t: 128 for t in synth.NTYPES}, seed=1, device=dev)
    x_dict = {k: f for k, f in enumerate(feats)}
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    torch.manual_seed(3)
    model = mag.REGNN(128, 64, 349, 2, 10.0, args.dropout, {k: 128 for k in x_dict}, 7,
                      use_norm="ln", self_loop_type=2).to(dev)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    n_paper = gd["counts"]["paper"]
    gen = torch.Generator(device=dev)
    gen.manual_seed(2)
    y_global = torch.full((gd["N"], 1), -1, dtype=torch.int64, device=dev)
    y_global[:n_paper, 0] = torch.randint(0, 349, (n_paper,), generator=gen, device=dev)
    sampler = NeighborSampler(rg, torch.arange(n_paper, device=dev), [25, 20], args.batch,
                              shuffle=True, seed=123, rank=rank, world_size=world)
    state = {"it": iter(sampler), "epoch": 0, "edges": 0}

    def step():
        try:
            batch = next(state["it"])
        except StopIteration:
            state["epoch"] += 1
            sampler.set_epoch(state["epoch"])
            state["it"] = iter(sampler)
            batch = next(state["it"])
        _, n_id, adjs = batch
        state["edges"] += sum(a.edge_index.shape[1] + a.size[1] for a in adjs)  # + self loops
        mag.train_step(model, opt, batch, x_dict, edge_type, node_type, local_node_idx,
                       y_global, world)

    torch.cuda.synchronize()
    log(f"[bench] ns: N={gd['N']:,} E={rg.E:,} built in {time.time() - t0:.1f}s; "
        f"{len(sampler)} batches/epoch/rank")
    return dict(step=step, edges_per_step=lambda: state["edges"], reset=lambda: state.update(edges=0),
                rg=rg, R=11, kernels=("spmm_fwd", "spmm_bwd"), convs=2, N=gd["N"], E=rg.E,
                ns=True)


def build_ns_infer(args, dev, t0):
    """mag/regnn_ns.py:348-369 layer-wise full-neighbour inference (2 x REGCNConv + LN + relu,
    out_lin), destination rows sharded over ranks with one all-gather per layer (strong
    scaling: the whole graph is one step's work, split across ranks)."""
    from regnn_hip import mag, synth
    from regnn_hip.graph import RelGraph
    from regnn_hip.inference import ShardedInference
    gd = synth.mag_like(args.scale, seed=0, device=dev)
    keep = gd["rel"] <= 7
    rg = RelGraph(gd["src"][keep], gd["dst"][keep], gd["N"], dev)
    edge_type = gd["rel"][keep].to(torch.int64) - 1
    del keep, gd["src"], gd["dst"], gd["rel"]
    node_type = gd["ntype"]
    offs = torch.tensor([gd["type_offsets"][t] for t in synth.NTYPES], device=dev)
    local_node_idx = torch.arange(gd["N"], device=dev) - offs[node_type]
    feats = synth.type_features(gd["counts"], {t: 128 for t in synth.NTYPES}, seed=1, device=dev)
    x_dict = {k: f for k, f in enumerate(feats)}
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    torch.manual_seed(3)
    model = mag.REGNN(128, 64, 349, 2, 10.0, 0.0, {k: 128 for k in x_dict}, 7,
                      use_norm="ln", self_loop_type=2).to(dev).eval()
    si = ShardedInference(model, rg, edge_type, node_type, local_node_idx, rank, world)
    del rg, edge_type
    torch.cuda.empty_cache()

    def step():
        si.run(x_dict, gather="argmax")

    torch.cuda.synchronize()
    log(f"[bench] ns_infer: N={gd['N']:,} rows {si.r0:,}..{si.r1:,} block E={si.block.E:,} "
        f"built in {time.time() - t0:.1f}s")
    return dict(step=step, edges_per_step=2 * si.block.E, rg=si.block, R=11,
                kernels=("spmm_fwd",), convs=2, N=gd["N"], E=si.block.E, scaling="strong")


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
    ap.add_argument("--workload", choices=["mag", "dblp", "acm", "imdb", "ns", "ns_infer"], default="mag")
    ap.add_argument("--scale", type=float, default=10.0)
    ap.add_argument("--batch", type=int, default=512, help="ns: target papers per rank")
    ap.add_argument("--dropout", type=float, default=0.5)
    ap.add_argument("--graph", choices=["auto", "on", "off"], default="auto",
                    help="capture the whole train step in a HIP graph and replay it "
                         "(auto: on for the launch-bound small graphs dblp/acm/imdb)")
    ap.add_argument("--dtype", choices=["fp32", "bf16"], default="fp32",
                    help="feature storage type of the REGCN workloads (mag, dblp); fp32 is the "
                         "reference's arithmetic and the default")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    rank, world, dev = setup_dist(args.gpus)
    from regnn_hip import profile

    w = build_workload(args, dev)
    rg = w["rg"]
    # (auto: capture the launch-bound single-GPU small graphs; with ranks > 1 the step holds an
    # RCCL all-reduce and runs eagerly)
    use_graph = args.graph == "on" or (args.graph == "auto" and world == 1 and
                                       args.workload in ("dblp", "acm", "imdb"))
    if use_graph and w.get("ns"):
        raise SystemExit("--graph: the sampled path has data-dependent shapes (not capturable)")
    for _ in range(args.warmup):
        w["step"]()
    torch.cuda.synchronize()
    if "reset" in w:
        w["reset"]()
    kstats = None
    run = w["step"]
    if use_graph:
        # per-op device times from eager profiled steps (events cannot sit inside a graph)
        profile.enable(True)
        for _ in range(min(args.steps, 10)):
            w["step"]()
        torch.cuda.synchronize()
        kstats = profile.summary()
        profile.enable(False)
        # capture one full train step (fwd + bwd + Adam) on a side stream, replay it K times
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):
                w["step"]()
        torch.cuda.current_stream().wait_stream(s)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            w["step"]()
        torch.cuda.synchronize()
        run = graph.replay
        run()
        torch.cuda.synchronize()

    if not use_graph:
        profile.enable(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if not use_graph:
        kstats = profile.summary()
        profile.enable(False)
    eps = w["edges_per_step"]
    edges = eps() if callable(eps) else eps * args.steps
    if world > 1:
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        e = torch.tensor([float(edges)], device=dev)
        dist.all_reduce(e, op=dist.ReduceOp.SUM)
        edges = float(e.item())
    ms = elapsed / args.steps * 1e3
    value = edges / elapsed if world > 1 else edges / elapsed

    # dominant HIP op (largest device time in the timed region) and its HBM roofline:
    # achieved = algorithmic bytes of its launches / their HIP-event durations
    cand = {k: v for k, v in kstats.items() if k in w["kernels"]}
    dom = max(cand, key=lambda k: cand[k][2])
    launches, mean_ms, total_ms, total_bytes = cand[dom]
    achieved = total_bytes / (total_ms / 1e3) / 1e9
    # HBM traffic per launch from the committed rocprofv3 PMC passes (tools/gpu_pmc.sh:
    # FETCH_SIZE and WRITE_SIZE in separate runs, calibrated on a 4 GiB copy), valid only for the
    # exact graph it was measured on
    traffic = None
    pmc = os.path.join(ROOT, "profiles", f"pmc_{args.workload}_{args.dtype}.json")
    if os.path.exists(pmc):
        with open(pmc) as f:
            rec = json.load(f)
        if rec.get("graph") == {"N": rg.n_dst, "E": rg.E} and rec.get("dtype") == args.dtype \
                and dom in rec:
            traffic = rec[dom]["bytes_per_launch"]

    desc = {
        "mag": f"REGCN 2-layer hidden=64 full-graph train step (input Linear, 2x REGraphConv "
               f"fwd+bwd, out_lin 349 classes, CE, Adam) on mag_like(scale={args.scale})",
        "dblp": "REGCN 2-layer hidden=64 full-graph train step on dblp_like (configs[1] shape)",
        "acm": "REGAT 2-layer hidden=64 heads [8,8,1] (last layer twice) train step on acm_like",
        "imdb": "REMixHop 2-layer p=[0,1,2] hidden=64 train step on imdb_like",
        "ns": f"mag/regnn_ns.py REGCN-NS train step (sample [25,20] x {args.batch} papers/rank, "
              f"group_input, 2x REGCNConv+LN, Adam, grad all-reduce) on mag_like(scale={args.scale})",
        "ns_infer": f"mag/regnn_ns.py layer-wise full-neighbour inference (2x REGCNConv+LN+relu, "
                    f"out_lin, argmax) on mag_like(scale={args.scale}), rows sharded over ranks, "
                    f"one all-gather per layer",
    }[args.workload]
    result = {
        "metric": "aggregated edges/sec per GPU (REGCN fwd+bwd, hidden=64); % HBM roofline",
        "value": value,
        "unit": "edges/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms,
        "higher_is_better": True,
        "scaling": w.get("scaling", "weak"),
        "vs_baseline": None,
        "dtype": args.dtype if args.workload in ("mag", "dblp") else "fp32",
        "data": "synthetic (seeded multi-relation graph of the BASELINE shape, random features/labels)",
        "config": {
            "workload": desc, "nodes": w["N"], "edges": w["E"], "relations": w["R"],
            "conv_applications_per_step": w["convs"], "hidden": 64,
            "parallelism": (f"data-parallel x{world} (RCCL grad all-reduce)" if w.get("ns")
                            else f"row-sharded x{world} (RCCL all-gather per layer)"
                            if w.get("scaling") == "strong" else
                            f"data-parallel x{world} over per-rank graph shards "
                            f"(RCCL grad all-reduce)"),
            "hip_graph": use_graph,
            # the last aggregation's backward gathers only the CSC edges into loss rows (the
            # output head's gradient is exactly zero elsewhere; ops.PRESCALE["prefix"])
            "last_layer_bwd_edges": (min(p.E for p in rg._prefix.values())
                                     if getattr(rg, "_prefix", None) else None),
        },
        "roofline": {
            "bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
            "launch_ms": mean_ms, "launches": launches,
            "algorithmic_bytes_per_launch": total_bytes / launches,
        },
        "kernels_ms": {k: round(v[1], 4) for k, v in kstats.items()},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        v, sample = cpu_baseline()
        result["cpu_baseline"] = {"value": v, "unit": "edges/s", "cores": 1, "kind": "port",
                                  "sample": sample + " (oracle/regnn_oracle.py numpy/scipy fp32)"}
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
