"""Benchmark — BASELINE.json metric "aggregated edges/sec per GPU (REGCN fwd+bwd, hidden=64);
% HBM roofline".

Default workload (`--workload ns`, BASELINE configs[4], the path the multi-GPU target is defined
on): the mag/regnn_ns.py REGCN neighbour-sampled training step on the ogbn-mag-scale synthetic
graph mag_like(10) (19.4 M nodes, 422 M edges, 7 edge types + 4 self-loop types), data-parallel
over ranks. One step = device sampler (batch 512 targets per rank, fan-out [25, 20]) ->
group_input -> 2 x REGCNConv (mean aggregation with the relation table, LayerNorm, ReLU,
dropout 0.5) -> out_lin (349 classes) -> log_softmax + nll -> backward -> one flat-bucket RCCL
all-reduce of the gradients -> Adam, captured as HIP graphs (regnn_hip.ns.NSTrainer: no host
synchronisation inside a step). The graph and features are replicated on every rank (weak
scaling: 512 targets per rank per step). value = aggregated edges (every sampled block's edges
incl. self loops, summed over ranks) / max-over-ranks time.

The top-level "roofline" is that of `value`'s own kernel, the fused NS model step
(regnn_nsm_step): algorithmic bytes (ns_step_bytes) / HIP-event time ("frac"), and the HBM bytes
rocprofv3 counted for the same kernels ("traffic", "frac_hbm", from profiles/pmc_ns_fp32.json
when it matches the kernel code and config).

At N = 1 the line also carries, on the same graph generator:
  * "full_batch": the full-graph REGCN training step on mag_like(10) (input Linear, 2 x
    REGraphConv fwd+bwd, out_lin, CE, Adam) -- the REGraphConv SpMM whose HBM roofline
    north_star gates (>= 40 %), with its own "roofline": "frac" from the rocprofv3-counted HBM
    bytes (profiles/pmc_mag_<dtype>.json, when it matches the kernel code), the SURVEY §8d
    algorithmic rate beside it as "frac_algorithmic" (it passes 1: Zipf hub rows hit in cache);
  * "cpu_baseline": oracle/cpu_ns.py, the same NS training step on the host cores (sampler
    spec, REGNN fwd+bwd as the reference composes it, nll, Adam; mag_like(1)), with the
    full-graph REGraphConv stack (oracle/cpu_regcn.py) under "full_batch".

Launch: python -m torch.distributed.run --nproc-per-node N bench.py --gpus N, or
    python bench.py --gpus N (starts that launcher itself as a child process), or
    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload ns|mag|dblp|acm|imdb|...]
"""
import argparse
import json
import os
import statistics
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
# Measured ceiling of a gather of B-byte rows at uniformly random indices out of an 8 GiB table
# (rows + 4-byte indices; tools/gather_probe.hip, profiles/r02_gather_probe.txt): the rate the
# SpMM's row gathers can reach on this part, below the sequential 8 TB/s.
GATHER_CEILING_GBS = {64: 2769.0, 128: 5106.0, 256: 5938.0, 512: 6008.0}
METRIC = "aggregated edges/sec per GPU (REGCN fwd+bwd, hidden=64); % HBM roofline"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def setup_dist(n):
    from regnn_hip.guard import pg_timeout
    if os.environ.get("REGNN_NS_FORCE_EXCHANGE") == "1" and n == 1:
        # one-rank rehearsal of the several-rank NS step structure (NSTrainer.rehearse_exchange)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=0, world_size=1, timeout=pg_timeout(),
                                device_id=torch.device("cuda", 0))
        return 0, 1, torch.device("cuda", 0)
    if n > 1 or int(os.environ.get("WORLD_SIZE", "1")) > 1:
        # RCCL ("nccl"); REGNN_DIST_BACKEND=gloo rehearses several ranks on one device. An
        # explicit timeout (REGNN_DIST_TIMEOUT, 600 s): a collective whose peer died errors out
        # instead of blocking forever; device_id binds the RCCL communicator to this rank's GPU
        backend = os.environ.get("REGNN_DIST_BACKEND", "nccl")
        local = int(os.environ.get("LOCAL_RANK", os.environ.get("RANK", "0")))
        local %= max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        kw = {"device_id": torch.device("cuda", local)} if backend == "nccl" else {}
        dist.init_process_group(backend, timeout=pg_timeout(), **kw)
        rank, world = dist.get_rank(), dist.get_world_size()
    else:
        rank, world, local = 0, 1, 0
        torch.cuda.set_device(local)
    return rank, world, torch.device("cuda", local)


def self_launch(n):
    """run this script under `python -m torch.distributed.run --nproc-per-node n` (127.0.0.1, a
    free port) as a child process; rank 0 prints the JSON line. Returns the child's exit code."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)]
    log(f"[bench] launching {n} ranks: {' '.join(cmd[1:])} {' '.join(sys.argv[1:])}")
    return subprocess.call(cmd + sys.argv[1:])


def _world():
    return (dist.get_rank(), dist.get_world_size()) if dist.is_initialized() else (0, 1)


def _full_graph(gd, dev):
    import dgl
    g = dgl.DGLGraph((gd["src"], gd["dst"]), num_nodes=gd["N"])
    return g, g.relgraph(dev), gd["rel"].to(torch.int64)


# ---------------------------------------------------------------------------------------------
# neighbour-sampled step (configs[4])
# ---------------------------------------------------------------------------------------------
def build_ns(args, dev, hidden=None):
    """mag/regnn_ns.py training step on the device engine (regnn_hip.ns.NSTrainer)."""
    from regnn_hip import mag, synth
    from regnn_hip.graph import RelGraph
    from regnn_hip.ns import NSTrainer
    t0 = time.time()
    rank, world = _world()
    gd = synth.mag_like(args.scale, seed=0, device=dev, zipf_s=args.zipf)         # replicated on every rank
    keep = gd["rel"] <= 7                                       # the 7 raw edge types, no loops
    rg = RelGraph(gd["src"][keep], gd["dst"][keep], gd["N"], dev)
    edge_type = gd["rel"][keep].to(torch.int64) - 1
    del keep, gd["src"], gd["dst"], gd["rel"]
    node_type = gd["ntype"]
    offs = torch.tensor([gd["type_offsets"][t] for t in synth.NTYPES], device=dev)
    local_node_idx = torch.arange(gd["N"], device=dev) - offs[node_type]
    feats = synth.type_features(gd["counts"], {t: 128 for t in synth.NTYPES}, seed=1, device=dev)
    x_dict = {k: f for k, f in enumerate(feats)}
    torch.manual_seed(3)
    hidden = hidden or args.hidden
    model = mag.REGNN(128, hidden, 349, 2, 10.0, args.dropout, {k: 128 for k in x_dict}, 7,
                      use_norm="ln", self_loop_type=2).to(dev)
    n_paper = gd["counts"]["paper"]
    gen = torch.Generator(device=dev)
    gen.manual_seed(2)
    y_global = torch.full((gd["N"], 1), -1, dtype=torch.int64, device=dev)
    y_global[:n_paper, 0] = torch.randint(0, 349, (n_paper,), generator=gen, device=dev)
    # Adam (mag/regnn_ns.py:495, lr 1e-3) as one flat-bucket launch (regnn_hip.ns.FlatAdam)
    tr = NSTrainer(model, None, rg, [25, 20], args.batch, torch.arange(n_paper, device=dev),
                   x_dict, edge_type, node_type, local_node_idx, y_global, 7, seed=123,
                   rank=rank, world=world, adam=dict(lr=1e-3))
    if os.environ.get("REGNN_NS_FORCE_EXCHANGE") == "1":
        tr.rehearse_exchange()
    torch.cuda.synchronize()
    log(f"[bench] ns: N={gd['N']:,} E={rg.E:,} built in {time.time() - t0:.1f}s; "
        f"{tr.steps_per_epoch()} steps/epoch/rank, capacities {tr.sampler.caps}")
    return tr, dict(N=gd["N"], E=rg.E, n_train=n_paper, rg=rg, edge_type=edge_type,
                    node_type=node_type, local=local_node_idx, x_dict=x_dict, model=model)


def run_ns_epoch(args, dev):
    """context line: one whole NS training epoch over the synthetic paper train
    split (steps_per_epoch steps, HIP-graph replays) plus the layer-wise full-neighbour
    inference pass the reference runs each epoch (mag/regnn_ns.py:348-369, 422-443), in seconds,
    next to mag/README.md:226-234 (448 s/epoch for the reference on 4 CPU cores, hidden 512,
    ogbn-mag). The fused step covers hidden 64; other widths run the autograd path."""
    from regnn_hip.inference import ShardedInference
    rank, world = _world()
    tr, info = build_ns(args, dev)
    steps = tr.steps_per_epoch()
    tr.capture(warmup=2)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tr.run_steps(steps)
    torch.cuda.synchronize()
    t_train = time.perf_counter() - t0
    model = info["model"].eval()
    si = ShardedInference(model, info["rg"], info["edge_type"], info["node_type"],
                          info["local"], rank, world)
    si.run(info["x_dict"], gather="argmax")          # warm-up (kernel selection)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    si.run(info["x_dict"], gather="argmax")
    torch.cuda.synchronize()
    t_inf = time.perf_counter() - t0
    return {"metric": "NS training epoch + full-neighbour inference (s)",
            "value": t_train + t_inf, "unit": "s", "n_gpus": world, "steps": steps,
            "warmup": 2, "ms_per_step": t_train / steps * 1e3, "higher_is_better": False,
            "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
            "data": "synthetic (seeded ogbn-mag-shaped graph)",
            "config": {"workload": f"mag_like(scale={args.scale}) NS epoch: {steps} steps of "
                                   f"{args.batch} papers x [25, 20], hidden {args.hidden}, "
                                   f"then layer-wise inference over every node",
                       "engine": "fused regnn_nsm_step" if tr.fused is not None else "module",
                       "train_s": t_train, "inference_s": t_inf,
                       "reference_context": "mag/README.md:226-234: 448.42 s per epoch, 4 CPU "
                                            "cores, hidden 512, real ogbn-mag"}}


def ns_step_bytes(sz, K, C, L=2, F=64, T=4, rel_slots=False, two_layer=True, adam_params=0,
                  pre_sums=False):
    """algorithmic HBM bytes of one fused NS model step (regnn_nsm_step) at the sampled sizes
    sz (regnn_ns_hop sizes: sz[h] = rows after h hops, sz[8 + h] = edges of hop h's block,
    self loops included): every row / index / feature byte a kernel must read or write once
    (per-block partial slabs are not counted: they are the reductions' own traffic).

    Two-layer step (re_nsm2.hip; n1 = layer 0's target rows, E1 its edges, n0 / E0 layer 1's):
      agg0      E1 x (K*4 gathered input row + 13 type / row / relation) + n1 x (T*K*4 per-type
                sums + 4*T counts + 4*F each for a, h0, P + 8*F gradient accumulators zeroed
                + 16 stats / ptr / inv); relation slots: + n1 x (K*4 self row + 4*(T+1) slots)
      head      E0 x 2 x (F*4 h0 row + 5) (aggregation, then the transposed pass) + E0 x 8*F
                (fixed-point accumulators) + n0 x 24 + 4*C*F + 4*F*F
      bwd0      n1 x (8*F accumulators + 4*F a + 4*F P + 12 stats / inv + T*K*4 per-type sums +
                4*T counts); relation slots: + n1 x (K*4 self row + 4*(T+1) slots); else
                + n1 x (T*K*4 Z + 4*T beta) and rel0's E1 x (K*4 + 13) + n1 x (T*K*4 + 4*T)
      Adam      24 B per parameter (p, m, v read and written) when it runs inside the step
    pre_sums (regnn_nsm_work.pre_sums): the sampler formed layer 0's per-type input sums ahead of
    the step (regnn_ns_hop_typed_sums); agg0 reads the n1 x (T*K*4 + 4*T + K*4 + 4*(T+1)) bytes of
    sums / counts / self rows / slots instead of gathering E1 input rows and writing them.
    The L-layer composed-map form (two_layer=False) keeps round 2's model."""
    f = 4 * F
    if two_layer and L == 2:
        n1, E1, n0, E0 = sz[1], sz[9], sz[0], sz[8]
        gather0 = 0 if pre_sums else E1 * (4 * K + 13)
        b = gather0 + n1 * (T * 4 * K + 4 * T + 3 * f + 2 * f + 16)
        b += E0 * 2 * (f + 5) + E0 * 2 * f + n0 * 24 + 4 * C * F + 4 * F * F
        b += n1 * (2 * f + f + f + 12 + T * 4 * K + 4 * T)
        if rel_slots:
            b += 2 * n1 * (4 * K + 4 * (T + 1))
        else:
            b += n1 * (T * 4 * K + 4 * T)
            b += E1 * (4 * K + 13) + n1 * (T * 4 * K + 4 * T)
        return b + 24 * adam_params
    n, E = sz[L - 1], sz[8 + L - 1]
    b = E * (4 * K + 13) + n * (T * 4 * K + 4 * T + 3 * f + 16)       # agg0
    if rel_slots:
        b += n * (4 * K + 4 * (T + 1))                                  # agg0: self rows, slots
        b += n * (T * 4 * K + 4 * K + 4 * (T + 1) + f + 4 * T + 4)      # bwd0
    else:
        b += n * (2 * T * 4 * K + f + 8 * T + 4)                        # bwd0
        b += E * (4 * K + 13) + n * (T * 4 * K + 4 * T)                 # rel0
    for l in range(1, L - 1):                                           # agg / agg_bwd
        h = L - 1 - l
        b += sz[8 + h] * (f + 5) + sz[h] * (4 * f + 20)
        b += sz[8 + h] * (2 * f + 5) + sz[h] * (f + 12)
    for l in range(L - 1):                                              # post_bwd
        b += sz[L - 1 - l] * (3 * f + 8)
    b += sz[8] * (f + 5) + sz[0] * (f + 24) + 4 * C * F                # head (layer L-1)
    b += sz[8] * (2 * f + 5) + sz[0] * (f + 12)                         # its agg_bwd
    return b


def ns_sums_bytes(sz, K, T):
    """Algorithmic HBM bytes of the sampler's outer-hop sums launch (regnn_ns_hop_typed_sums,
    hop 1 of the two-layer step; n1 = sizes[1] rows, E1 = sizes[9] slots incl. self loops):
      per row    n_id + ptr pair 12, scnt + inv 8, and its outputs: T*K*4 sums, 4*T counts,
                 K*4 self row, 4*(T+1) slot relations
      per slot   idx 4 + etype 1 + node type 4 + table row 8 read, the raw input row K*4
                 gathered, and the edge meta 13 (relation 1, source type 4, table row 8) written"""
    n1, E1 = sz[1], sz[9]
    return E1 * (4 + 1 + 4 + 8 + 4 * K + 13) + n1 * (12 + 8 + T * 4 * K + 4 * T + 4 * K + 4 * (T + 1))


def pmc_traffic_sums():
    """HBM bytes per sums launch from the same committed PMC summary, or (None, reason)."""
    from regnn_hip.build import NS_SUMS_SOURCES, kernel_hash
    path = os.path.join(ROOT, "profiles", "pmc_ns_fp32.json")
    if not os.path.exists(path):
        return None, "no PMC summary committed"
    with open(path) as f:
        rec = json.load(f)
    if "ns_sums" not in rec:
        return None, "PMC summary has no sums record"
    if rec.get("sums_code_hash") != kernel_hash(NS_SUMS_SOURCES):
        return None, "PMC summary is for other kernel code (stale: re-run tools/gpu_pmc_ns.sh)"
    return rec["ns_sums"]["bytes_per_launch"], "ok"


def run_ns(args, dev):
    from regnn_hip import profile
    from regnn_hip.guard import Guard
    rank, world = _world()
    # every stage that may fail on one rank ends on an agreement of all ranks (regnn_hip.guard):
    # a failure anywhere exits every rank non-zero instead of leaving peers in a collective
    guard = Guard(world)
    tr, info = guard.stage("build the NS trainer (graph, features, model, sampler)",
                           lambda: build_ns(args, dev))
    # per-op device times from eager profiled steps (events cannot sit inside a graph)
    for _ in range(max(1, args.warmup)):
        tr.guarded_step(guard)
    profile.enable(True)
    nsm_bytes = []
    for _ in range(5):
        tr.guarded_step(guard)
        if tr.fused is not None:
            nsm_bytes.append(ns_step_bytes(
                tr.sampler.sizes.cpu().tolist(), 128, 349, rel_slots=bool(tr.fused.P.rel_slots),
                two_layer=tr.fused.two_layer,
                adam_params=tr.flat.numel() if tr.adam_fused else 0,
                pre_sums=bool(tr.fused.W.pre_sums)))
    torch.cuda.synchronize()
    kstats = profile.summary()
    profile.enable(False)
    use_graph = args.graph != "off"
    capture_s = None
    if use_graph:
        t_cap = time.time()
        guard.stage("capture the step graphs", lambda: tr.capture(warmup=2))
        capture_s = time.time() - t_cap
        log(f"[bench] ns: captured the step graphs in {capture_s:.1f}s (lookahead {tr.ahead})")
        run_k = tr.run_steps               # step pairs as one graph replay where they fit
    else:
        def run_k(k):
            for _ in range(k):
                tr.step()
    run_k(args.warmup)
    torch.cuda.synchronize()
    e0 = tr.edges_total()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run_k(args.steps)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    edges = tr.edges_total() - e0
    loss = float(tr.loss)
    if world > 1:
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        e = torch.tensor([float(edges)], device=dev)
        dist.all_reduce(e, op=dist.ReduceOp.SUM)
        edges = float(e.item())
    ms = elapsed / args.steps * 1e3
    exchanged = world > 1 or tr._force_exchange
    if not exchanged:
        exchange = None
    elif not use_graph:
        exchange = "eager all-reduce after each step"
    elif tr.exchange_in_graph:
        exchange = "all-reduce captured in the step graph"
    else:
        exchange = "eager all-reduce between graphs"
    if exchange and tr._xsplit and tr._early_ok:
        exchange += (f"; the {tr.n_early} gradients final after layer 1's transposed pass "
                     "all-reduced on a comm stream under layer 0's backward")
    res = {
        "metric": METRIC,
        "value": edges / elapsed,
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
            "workload": (f"mag/regnn_ns.py REGCN neighbour-sampled train step: device sampler "
                         f"{args.batch} papers/rank x fan-out [25, 20], group_input, 2x REGCNConv "
                         f"(hidden {args.hidden}, mean, relation table, LN, ReLU, dropout "
                         f"{args.dropout}), out_lin 349, nll, backward, "
                         + (f"{dist.get_backend() if dist.is_initialized() else ''} flat-bucket "
                            f"grad all-reduce ({exchange}), " if exchange else "")
                         + f"Adam; mag_like(scale={args.scale}) replicated per rank"),
            "nodes": info["N"], "edges": info["E"], "relations": 11, "hidden": args.hidden,
            "batch_per_rank": args.batch, "global_batch": args.batch * world,
            "fanout": [25, 20], "parallelism": f"dp{world}",
            "grad_exchange": exchange,
            "lookahead": tr.ahead,
            "hip_graph": use_graph, "lookahead": tr.ahead, "capture_s": capture_s,
            "aggregated_edges_per_step_per_rank": edges / world / args.steps,
            "final_loss": loss,
        },
        "ns_kernels_ms": {k: round(v[1], 4) for k, v in kstats.items()},
    }
    res["config"]["engine"] = "fused regnn_nsm_step" if tr.fused is not None else "module"
    if "nsm_step" in kstats and nsm_bytes:
        # the roofline of `value`'s own kernel: the fused model step (regnn_nsm_step), its
        # algorithmic bytes at the profiled steps' sampled sizes (ns_step_bytes) / its HIP-event
        # time; HBM bytes from the committed rocprofv3 FETCH_SIZE + WRITE_SIZE summary of the
        # same kernels (profiles/pmc_ns_fp32.json) when it matches this kernel code and config
        launches, mean_ms, total_ms, _ = kstats["nsm_step"]
        b = statistics.mean(nsm_bytes)
        ach = b / (mean_ms / 1e3) / 1e9
        traffic, pmc_status = pmc_traffic_ns(args)
        hbm = None if traffic is None else traffic / (mean_ms / 1e3) / 1e9
        res["roofline"] = {"bound": "hbm", "kernel": f"regnn_nsm_step ({tr.fused.launches()} "
                                                     f"launches: {', '.join(tr.fused.kernels())})",
                           "workload": "ns step (value)", "achieved": ach,
                           "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
                           "traffic": traffic, "achieved_hbm": hbm,
                           "frac_hbm": None if hbm is None else hbm / HBM_PEAK_GBS,
                           "pmc": pmc_status, "launch_ms": mean_ms,
                           "profiled_launches": launches, "algorithmic_bytes_per_launch": b,
                           "note": "algorithmic bytes: bench.ns_step_bytes (DESIGN.md §4b); the "
                                   "step is latency-bound (dependent phases), not byte-bound"}
    if "ns_typed_sums" in kstats and tr.fused is not None:
        # the sampler's one heavy launch (layer 0's input gather, G steps ahead on the second
        # stream): its own roofline, bytes at the mean of every sampled slot's sizes
        launches, mean_ms, _, _ = kstats["ns_typed_sums"]
        b = statistics.mean(ns_sums_bytes(sl.sizes.cpu().tolist(), 128, tr.fused.P.n_types)
                            for sl in tr.slots)
        ach = b / (mean_ms / 1e3) / 1e9
        traffic, pmc_status = pmc_traffic_sums()
        hbm = None if traffic is None else traffic / (mean_ms / 1e3) / 1e9
        res["sampler_roofline"] = {
            "bound": "hbm", "kernel": "regnn_ns_hop_typed_sums (ns_sample_sums_kernel)",
            "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
            "traffic": traffic, "achieved_hbm": hbm,
            "frac_hbm": None if hbm is None else hbm / HBM_PEAK_GBS, "pmc": pmc_status,
            "launch_ms": mean_ms, "profiled_launches": launches, "algorithmic_bytes_per_launch": b,
            "note": "eager profiled steps: the launch shares the GPU with the model step; "
                    "algorithmic bytes: bench.ns_sums_bytes (every slot's raw row gathered once)"}
    cand = {k: v for k, v in kstats.items() if k in ("ns_spmm_fwd", "ns_spmm_bwd")}
    if cand:
        dom = max(cand, key=lambda k: cand[k][2])
        launches, mean_ms, total_ms, total_bytes = cand[dom]
        ach = total_bytes / (total_ms / 1e3) / 1e9
        res["roofline"] = {"bound": "hbm", "kernel": dom, "workload": "ns step (module path)",
                           "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                           "frac": ach / HBM_PEAK_GBS, "traffic": None, "launch_ms": mean_ms,
                           "algorithmic_bytes_per_launch": total_bytes / launches}
    del tr
    torch.cuda.empty_cache()
    return res


# ---------------------------------------------------------------------------------------------
# full-graph workloads (configs[0..3] shapes and the mag-10x roofline step)
# ---------------------------------------------------------------------------------------------
def build_full(args, dev, wl):
    """-> dict(step=callable, edges_per_step, rg, kernels, ...) for a full-graph workload."""
    from regnn_hip import mag, nets, ops, synth
    t0 = time.time()
    rank, world = _world()
    gen = torch.Generator(device=dev)
    gen.manual_seed(2)
    torch.manual_seed(3)
    if wl in ("mag", "dblp"):
        if wl == "mag":
            gd = synth.mag_like(args.scale, seed=0, device=dev, zipf_s=args.zipf)
            feats = synth.type_features(gd["counts"], {t: 128 for t in synth.NTYPES}, seed=1,
                                        device=dev, kind="mag")
            # a random train split at ogbn-mag's train fraction (629,571 of 736,389 papers),
            # its rows renumbered first once (data.loss_rows_first): head_ce's loss-row prefix
            from regnn_hip import data
            n_paper = gd["counts"]["paper"]
            split_gen = torch.Generator(device=dev)
            split_gen.manual_seed(5)
            train = torch.randperm(n_paper, generator=split_gen, device=dev)
            train = train[:int(round(n_paper * 629_571 / 736_389))]
            perm, inv = data.loss_rows_first(gd["N"], train, n_paper)
            gd["src"], gd["dst"] = inv[gd["src"]], inv[gd["dst"]]
            feats[0] = feats[0][perm[:n_paper]].contiguous()
            del perm, inv
            n_classes, train_nodes = 349, train.numel()
        else:
            gd = synth.dblp_like(seed=0, device=dev)
            feats = synth.type_features(gd["counts"], synth.DBLP_DIMS, seed=1, device=dev,
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
        gd = synth.acm_like(seed=0, device=dev)
        feats = synth.type_features(gd["counts"], synth.ACM_DIMS, seed=1, device=dev,
                                    kind="target")
        n_classes, train_nodes = 3, gd["counts"]["P"]
        g, rg, e_feat = _full_graph(gd, dev)
        net = nets.REGAT(g, gd["R"], 100.0, 2, 64, 64, n_classes, [8, 8, 1], F.elu, args.dropout,
                         args.dropout, 0.01, False, [f.shape[1] for f in feats]).to(dev)
        convs, kern = 3, ("spmm_heads_fwd", "spmm_heads_bwd", "gat_softmax_fwd",
                          "gat_softmax_bwd")
    elif wl == "gat":
        # the fused GAT path where bandwidth is the limit: one REGATConv
        # layer (heads 8, out 64, relation bias, LeakyReLU 0.01) forward + backward on the
        # ogbn-mag-shaped graph mag_like(scale); ft rows are 8 x 64 fp32 = 2 KiB
        from layer import REGATConv
        gd = synth.mag_like(args.scale, seed=0, device=dev, zipf_s=args.zipf)
        g, rg, e_feat = _full_graph(gd, dev)
        conv = REGATConv(gd["R"], 100.0, 64, 64, 8, 0.0, 0.0, 0.01).to(dev).eval()
        x = torch.randn(gd["N"], 64, generator=gen, device=dev)
        gout = torch.randn(gd["N"], 8, 64, generator=gen, device=dev)
        params = list(conv.parameters())

        def step():
            y = conv(g, x, e_feat)
            y.backward(gout)
            for p_ in params:
                p_.grad = None

        torch.cuda.synchronize()
        log(f"[bench] gat: N={gd['N']:,} E={rg.E:,} R={gd['R']} built in {time.time() - t0:.1f}s")
        return dict(step=step, edges_per_step=rg.E, rg=rg, R=gd["R"],
                    kernels=("gat_fused_fwd", "spmm_heads_bwd", "gat_softmax_bwd",
                             "gat_attn_lse"), convs=1, N=rg.n_dst, E=rg.E, train_nodes=0)
    elif wl == "gatv2":
        # one REGATv2Conv layer (heads 8, out 64, relation bias, LeakyReLU 0.01) forward +
        # backward on mag_like(scale): the GATv2 score SDDMM, the per-destination edge softmax
        # and the per-head aggregation; Zipf hub rows take the long-segment plan
        from layer import REGATv2Conv
        gd = synth.mag_like(args.scale, seed=0, device=dev, zipf_s=args.zipf)
        g, rg, e_feat = _full_graph(gd, dev)
        conv = REGATv2Conv(gd["R"], 100.0, 64, 64, 8, 0.0, 0.0, 0.01).to(dev).train()
        x = torch.randn(gd["N"], 64, generator=gen, device=dev)
        gout = torch.randn(gd["N"], 8, 64, generator=gen, device=dev)
        params = list(conv.parameters())

        def step():
            y = conv(g, x, e_feat)
            y.backward(gout)
            for p_ in params:
                p_.grad = None

        torch.cuda.synchronize()
        log(f"[bench] gatv2: N={gd['N']:,} E={rg.E:,} R={gd['R']} built in {time.time() - t0:.1f}s; "
            f"long rows csr={rg.csr_plan.n_long} csc={rg.csc_plan.n_long}")
        return dict(step=step, edges_per_step=rg.E, rg=rg, R=gd["R"],
                    kernels=("gatv2_score_fwd", "gatv2_score_bwd", "edge_softmax_fwd",
                             "edge_softmax_bwd", "spmm_heads_fwd", "spmm_heads_bwd"),
                    convs=1, N=rg.n_dst, E=rg.E, train_nodes=0)
    elif wl == "imdb":
        gd = synth.imdb_like(seed=0, device=dev)
        feats = synth.type_features(gd["counts"], synth.IMDB_DIMS, seed=1, device=dev,
                                    kind="target")
        n_classes, train_nodes = 3, gd["counts"]["M"]
        g, rg, e_feat = _full_graph(gd, dev)
        net = nets.REMixHop(g, gd["R"], 100.0, 64, 64, n_classes, 2, [f.shape[1] for f in feats],
                            input_dropout=args.dropout, activation=F.elu).to(dev)
        convs, kern = 4, ("spmm_fwd", "spmm_bwd")        # 2 live hops x 2 layers
    else:
        raise ValueError(wl)
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
            mag.flat_grad_allreduce(params, world)      # replicas: averaged gradients
        opt.step()

    torch.cuda.synchronize()
    log(f"[bench] {wl}: N={gd['N']:,} E={rg.E:,} R={gd['R']} built in {time.time() - t0:.1f}s; "
        f"long rows csr={rg.csr_plan.n_long} csc={rg.csc_plan.n_long}")
    return dict(step=step, edges_per_step=convs * rg.E, rg=rg, R=gd["R"], kernels=kern,
                convs=convs, N=rg.n_dst, E=rg.E, train_nodes=train_nodes)


def pmc_traffic(wl, dtype, rg, op):
    """HBM bytes per launch of `op` from the committed rocprofv3 PMC summary
    (tools/gpu_pmc2.sh: FETCH_SIZE / WRITE_SIZE in separate passes, copy-calibrated), or
    (None, reason) when it was measured on another graph, dtype or kernel code."""
    from regnn_hip.build import kernel_hash
    path = os.path.join(ROOT, "profiles", f"pmc_{wl}_{dtype}.json")
    if not os.path.exists(path):
        return None, "no PMC summary committed"
    with open(path) as f:
        rec = json.load(f)
    if rec.get("graph") != {"N": rg.n_dst, "E": rg.E} or rec.get("dtype") != dtype:
        return None, "PMC summary is for another graph / dtype"
    if rec.get("code_hash") != kernel_hash():
        return None, "PMC summary is for other kernel code (stale: re-run tools/gpu_pmc2.sh)"
    if op not in rec:
        return None, f"PMC summary has no {op}"
    return rec[op]["bytes_per_launch"], "ok"


def pmc_traffic_ns(args):
    """HBM bytes per fused NS model step from the committed rocprofv3 PMC summary
    (tools/gpu_pmc_ns.sh: FETCH_SIZE / WRITE_SIZE of the regnn::nsm kernels, separate passes,
    copy-calibrated), or (None, reason) when it was measured on other kernel code or config."""
    from regnn_hip.build import NS_PMC_SOURCES, kernel_hash
    path = os.path.join(ROOT, "profiles", "pmc_ns_fp32.json")
    if not os.path.exists(path):
        return None, "no PMC summary committed"
    with open(path) as f:
        rec = json.load(f)
    want = {"scale": args.scale, "batch": args.batch, "fanout": [25, 20], "hidden": args.hidden,
            "dropout": args.dropout}
    if rec.get("config") != want:
        return None, f"PMC summary is for another config ({rec.get('config')})"
    if rec.get("code_hash") != kernel_hash(NS_PMC_SOURCES):
        return None, "PMC summary is for other kernel code (stale: re-run tools/gpu_pmc_ns.sh)"
    return rec["nsm_step"]["bytes_per_launch"], "ok"


def run_full(args, dev, wl):
    from regnn_hip import profile
    rank, world = _world()
    w = build_full(args, dev, wl)
    use_graph = args.graph == "on" or (args.graph == "auto" and world == 1 and
                                       wl in ("dblp", "acm", "imdb"))
    for _ in range(args.warmup):
        w["step"]()
    torch.cuda.synchronize()
    kstats = None
    run = w["step"]
    if use_graph:
        profile.enable(True)
        for _ in range(min(args.steps, 10)):
            w["step"]()
        torch.cuda.synchronize()
        kstats = profile.summary()
        profile.enable(False)
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
    edges = w["edges_per_step"] * args.steps
    if world > 1:
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        edges *= world
    rg = w["rg"]
    # dominant HIP op (largest device time in the timed region) and its HBM roofline:
    # achieved = algorithmic bytes of its launches / their HIP-event durations
    cand = {k: v for k, v in kstats.items() if k in w["kernels"]}
    dom = max(cand, key=lambda k: cand[k][2])
    launches, mean_ms, total_ms, total_bytes = cand[dom]
    achieved = total_bytes / (total_ms / 1e3) / 1e9
    traffic, pmc_status = pmc_traffic(wl, args.dtype, rg, dom)
    hbm = None if traffic is None else traffic / (mean_ms / 1e3) / 1e9
    out = {
        "value": edges / elapsed, "ms_per_step": elapsed / args.steps * 1e3,
        "dtype": args.dtype if wl in ("mag", "dblp") else "fp32",
        "config": {"workload": {
            "mag": f"REGCN 2-layer hidden=64 full-graph train step (input Linear, 2x REGraphConv "
                   f"fwd+bwd, out_lin 349 classes, CE, Adam) on mag_like(scale={args.scale})",
            "dblp": "REGCN 2-layer hidden=64 full-graph train step on dblp_like (configs[1])",
            "acm": "REGAT 2-layer hidden=64 heads [8,8,1] (last layer twice) on acm_like",
            "imdb": "REMixHop 2-layer p=[0,1,2] hidden=64 on imdb_like",
            "gat": f"REGATConv heads 8 x 64, relation bias, fwd (fused scores + softmax + SpMM) "
                   f"+ bwd on mag_like(scale={args.scale}, zipf_s={args.zipf})",
            "gatv2": f"REGATv2Conv heads 8 x 64, relation bias, fwd (GATv2 score SDDMM, edge "
                     f"softmax, per-head SpMM) + bwd on mag_like(scale={args.scale}, "
                     f"zipf_s={args.zipf})"}[wl],
            "nodes": w["N"], "edges": w["E"], "relations": w["R"],
            "conv_applications_per_step": w["convs"], "hidden": 64, "hip_graph": use_graph,
            "label_rows": (f"{w['train_nodes']:,} train rows: a seeded random 85.5 % of the "
                           f"papers (ogbn-mag's train fraction), renumbered first once "
                           f"(data.loss_rows_first)" if wl == "mag" else
                           f"the first {w['train_nodes']:,} nodes (the target type)"),
            "last_layer_bwd_edges": (min(p.E for p in rg._prefix.values())
                                     if getattr(rg, "_prefix", None) else None)},
        # frac is a real fraction of the HBM peak: the rocprofv3-counted bytes per launch
        # (FETCH_SIZE + WRITE_SIZE, copy-calibrated) over the launch time when the committed PMC
        # summary matches this graph / dtype / kernel code. The SURVEY §8d algorithmic bytes
        # charge every gathered row to HBM; on the Zipf graphs the hub source rows hit in L2 /
        # the Infinity Cache, so that rate can pass 8 TB/s (kept as achieved_algorithmic /
        # frac_algorithmic, not a fraction of anything)
        "roofline": {
            "bound": "hbm", "kernel": dom, "workload": f"full_batch {wl}",
            "achieved": hbm if hbm is not None else achieved, "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": (hbm if hbm is not None else achieved) / HBM_PEAK_GBS,
            "frac_basis": ("rocprofv3 HBM bytes (FETCH_SIZE + WRITE_SIZE) per launch" if hbm is not None
                           else f"algorithmic bytes (PMC: {pmc_status})"),
            "traffic": traffic,
            "achieved_algorithmic": achieved, "frac_algorithmic": achieved / HBM_PEAK_GBS,
            "achieved_hbm": hbm, "frac_hbm": None if hbm is None else hbm / HBM_PEAK_GBS,
            "pmc": pmc_status, "launch_ms": mean_ms, "launches": launches,
            "algorithmic_bytes_per_launch": total_bytes / launches,
            "gather_ceiling": _gather_ceiling(wl, args.dtype, hbm)},
        "kernels_ms": {k: round(v[1], 4) for k, v in kstats.items()},
    }
    del w
    torch.cuda.empty_cache()
    return out


def _gather_ceiling(wl, dtype, hbm):
    """The random row-gather ceiling for the SpMM's rows (hidden 64: 256 B fp32, 128 B bf16)."""
    if wl not in ("mag", "dblp"):
        return None
    row = 64 * (2 if dtype == "bf16" else 4)
    c = GATHER_CEILING_GBS[row]
    return {"row_bytes": row, "GB/s": c, "source": "profiles/r02_gather_probe.txt",
            "hbm_over_ceiling": None if hbm is None else hbm / c}


def build_ns_infer(args, dev):
    """mag/regnn_ns.py:348-369 layer-wise full-neighbour inference, rows sharded over ranks."""
    from regnn_hip import mag, synth
    from regnn_hip.graph import RelGraph
    from regnn_hip.inference import ShardedInference
    rank, world = _world()
    gd = synth.mag_like(args.scale, seed=0, device=dev, zipf_s=args.zipf)
    keep = gd["rel"] <= 7
    rg = RelGraph(gd["src"][keep], gd["dst"][keep], gd["N"], dev)
    edge_type = gd["rel"][keep].to(torch.int64) - 1
    del keep, gd["src"], gd["dst"], gd["rel"]
    node_type = gd["ntype"]
    offs = torch.tensor([gd["type_offsets"][t] for t in synth.NTYPES], device=dev)
    local_node_idx = torch.arange(gd["N"], device=dev) - offs[node_type]
    feats = synth.type_features(gd["counts"], {t: 128 for t in synth.NTYPES}, seed=1, device=dev)
    x_dict = {k: f for k, f in enumerate(feats)}
    torch.manual_seed(3)
    model = mag.REGNN(128, 64, 349, 2, 10.0, 0.0, {k: 128 for k in x_dict}, 7,
                      use_norm="ln", self_loop_type=2).to(dev).eval()
    si = ShardedInference(model, rg, edge_type, node_type, local_node_idx, rank, world)
    del rg, edge_type
    torch.cuda.empty_cache()
    return si, gd["N"], x_dict


# ---------------------------------------------------------------------------------------------
# CPU baseline: torch.sparse CSR restatement on the host cores
# ---------------------------------------------------------------------------------------------
def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(scale=1.0, reps=10, warm=3):
    """oracle/cpu_regcn.py REGraphConv x2 fwd+bwd (hidden 64, fp32) on mag_like(scale) and the
    DBLP shape, torch.set_num_threads(host share), median of `reps` after `warm` warm-ups."""
    from oracle import cpu_regcn as C
    from regnn_hip import synth
    threads = int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    out = {}
    try:
        for name, gd in (("dblp_like", synth.dblp_like(seed=0, device="cpu")),
                         (f"mag_like({scale:g})", synth.mag_like(scale, seed=0, device="cpu"))):
            g = C.CsrGraph(gd["src"], gd["dst"], gd["N"])
            rel = C.rel_csr_of(g, gd["rel"].to(torch.int64).numpy())
            del gd["src"], gd["dst"]
            x = torch.randn(gd["N"], 64, generator=torch.Generator().manual_seed(0))
            ws = [torch.full((gd["R"], 1), 0.01) for _ in range(2)]
            layers = [C.REGraphConvCPU(100.0) for _ in range(2)]
            times = []
            for i in range(warm + reps):
                t0 = time.perf_counter()
                C.regcn_stack_step(g, layers, x, rel, ws)
                if i >= warm:
                    times.append(time.perf_counter() - t0)
            t = statistics.median(times)
            out[name] = {"edges_per_s": 2 * g.E / t, "ms_per_step": t * 1e3, "N": gd["N"],
                         "E": g.E}
            del g, rel, x
    finally:
        torch.set_num_threads(prev)
    return out, threads


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # default: 160 timed steps for the NS step (20 lookahead groups of 8: a steadier figure than
    # 2.5 groups), 20 for the full-graph workloads and the full_batch leg
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=["ns", "mag", "dblp", "acm", "imdb", "gat", "gatv2",
                                           "ns_infer", "ns_epoch"], default="ns")
    ap.add_argument("--hidden", type=int, default=64, help="ns / ns_epoch: hidden width")
    ap.add_argument("--zipf", type=float, default=1.1,
                    help="mag_like destination skew (1.1: ogbn-mag-like hubs; 0: uniform)")
    ap.add_argument("--scale", type=float, default=10.0)
    ap.add_argument("--batch", type=int, default=512, help="ns: target papers per rank")
    ap.add_argument("--dropout", type=float, default=0.5)
    ap.add_argument("--graph", choices=["auto", "on", "off"], default="auto",
                    help="HIP-graph capture of the step (auto: on for ns and the launch-bound "
                         "small graphs dblp/acm/imdb)")
    ap.add_argument("--dtype", choices=["fp32", "bf16"], default="fp32",
                    help="feature storage type of the full-graph REGCN workloads (mag, dblp)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-full-batch", action="store_true",
                    help="ns at N=1: skip the full-graph roofline leg")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # `python bench.py --gpus N` without a launcher: start the N ranks as a child
        # torch.distributed.run (this process never touches the GPU) and exit with its code
        sys.exit(self_launch(args.gpus))

    rank, world, dev = setup_dist(args.gpus)
    explicit_steps = args.steps is not None
    if not explicit_steps:
        args.steps = 160 if args.workload == "ns" else 20
    if args.workload == "ns":
        result = run_ns(args, dev)
        if world == 1 and not args.no_full_batch:
            # the full-graph REGraphConv step: north_star's SpMM roofline gate, under its own key
            if not explicit_steps:
                args.steps = 20
            result["full_batch"] = run_full(args, dev, "mag")
    elif args.workload == "ns_infer":
        result = run_other_ns_infer(args, dev)
    elif args.workload == "ns_epoch":
        result = run_ns_epoch(args, dev)
    else:
        fb = run_full(args, dev, args.workload)
        result = {"metric": METRIC, "value": fb["value"], "unit": "edges/s", "n_gpus": world,
                  "steps": args.steps, "warmup": args.warmup, "ms_per_step": fb["ms_per_step"],
                  "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
                  "dtype": fb["dtype"],
                  "data": "synthetic (seeded multi-relation graph of the BASELINE shape, "
                          "random features/labels)",
                  "config": dict(fb["config"], parallelism=f"replicas x{world} (averaged grads)"),
                  "roofline": fb["roofline"], "kernels_ms": fb["kernels_ms"]}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cb, threads = cpu_baseline()
        mag_key = [k for k in cb if k.startswith("mag_like")][0]
        full = {
            "value": cb[mag_key]["edges_per_s"], "unit": "edges/s", "cores": threads,
            "kind": "port", "cpu_model": _cpu_model(),
            "sample": (f"oracle/cpu_regcn.py (torch.sparse CSR fwd+bwd of REGraphConv x2, "
                       f"hidden 64, fp32) on {mag_key} N={cb[mag_key]['N']:,} "
                       f"E={cb[mag_key]['E']:,}; median of 10 after 3 warm-ups"),
            "dblp_like": cb["dblp_like"], mag_key: cb[mag_key]}
        if args.workload == "ns":
            # the workload `value` measures: the NS training step on the host cores
            from oracle import cpu_ns
            t, e, info = cpu_ns.step_baseline(scale=1.0, steps=10, warm=3, threads=threads)
            result["cpu_baseline"] = {
                "value": e / t, "unit": "edges/s", "cores": info["threads"], "kind": "port",
                "cpu_model": _cpu_model(), "ms_per_step": t * 1e3,
                "aggregated_edges_per_step": e,
                "value_aggregated_edges_per_step": result["config"].get(
                    "aggregated_edges_per_step_per_rank"),
                "sample": (f"oracle/cpu_ns.py: the NS training step (the sampler spec, REGNN "
                           f"regcn/LN fwd+bwd with index_add scatter as the reference composes "
                           f"it, nll, Adam) on mag_like(1) N={info['N']:,} E={info['E']:,}, "
                           f"batch {info['batch']} x {info['sizes']}, hidden 64, 349 classes, "
                           f"dropout 0.5; median of 10 steps after 3 warm-ups. Same generator "
                           f"at 1/10 the size of value's mag_like({args.scale:g}): "
                           f"{e:,.0f} aggregated edges per step here against "
                           f"{result['config'].get('aggregated_edges_per_step_per_rank', 0):,.0f} "
                           f"per rank-step in value (both rates are per aggregated edge)"),
                "full_batch": full}
        else:
            result["cpu_baseline"] = full
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


def run_other_ns_infer(args, dev):
    """strong scaling: the whole graph's layer-wise inference is one step, rows split over ranks."""
    rank, world = _world()
    si, N, x_dict = build_ns_infer(args, dev)
    for _ in range(args.warmup):
        si.run(x_dict, gather="argmax")
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        si.run(x_dict, gather="argmax")
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    edges = 2 * si.block.E * args.steps
    if world > 1:
        e = torch.tensor([float(edges)], device=dev)
        dist.all_reduce(e, op=dist.ReduceOp.SUM)
        edges = float(e.item())
    return {"metric": METRIC, "value": edges / elapsed, "unit": "edges/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "fp32",
            "data": "synthetic (seeded ogbn-mag-shaped graph)",
            "config": {"workload": f"mag/regnn_ns.py layer-wise full-neighbour inference "
                                   f"(2x REGCNConv+LN+relu, out_lin, argmax) on "
                                   f"mag_like(scale={args.scale}), rows sharded over ranks",
                       "nodes": N, "parallelism": f"row-sharded x{world}"}}


if __name__ == "__main__":
    main()
