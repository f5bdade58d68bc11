"""The data-parallel NS step with two ranks on the box's one GPU (gloo standing in for RCCL, which
cannot run two ranks on one device): the pipelined trainer with world = 2 captured as
two HIP graphs with the flat-bucket all-reduce between them (what `bench.py --gpus N` runs
under torch.distributed.run), then eager steps. Both ranks must hold bit-identical parameters
after every step (the all-reduced gradient and the same Adam), train on different batches, and
see finite losses (mag/regnn_ns.py:392-420 with DistributedDataParallel's contract)."""
import os
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _worker(rank, world, port, q):
    try:
        import torch.distributed as dist
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        sys.path.insert(0, HERE)
        sys.path.insert(0, os.path.join(os.path.dirname(HERE), "re-gnn_amd"))
        from test_gpu_ns_engine import _mag
        from regnn_hip.ns import NSTrainer
        d = _mag(0.002, seed=8, F=128, hidden=64, classes=13, dropout=0.3)
        tr = NSTrainer(d["model"](5), None, d["rg"], [6, 4], 64,
                       torch.arange(d["n_paper"], device="cuda"), d["x_dict"], d["edge_type"],
                       d["node_type"], d["local"], d["y"], 7, seed=9, rank=rank, world=world,
                       adam=dict(lr=1e-2))
        assert tr.pipelined
        tr.capture(warmup=1)
        out = {"loss": [], "params": [], "targets": []}
        for i in range(6):
            (tr.replay if i < 4 else tr.step)()
            torch.cuda.synchronize()
            s = tr.sampler
            out["loss"].append(float(tr.loss))
            # numpy: pickled by value (torch tensors would travel as shared-memory handles that
            # die with this process)
            out["params"].append(tr.pflat.detach().cpu().numpy().copy())
            out["targets"].append(s.n_id[:int(s.sizes[0])].cpu().numpy().copy())
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, out))
    except Exception as e:                      # surface the failure in the parent
        q.put((rank, repr(e)))


def test_ns_dp_two_ranks_one_gpu():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (os.getpid() % 1000)
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for r in (0, 1):
        assert not isinstance(res[r], str), f"rank {r}: {res[r]}"
    a, b = res[0], res[1]
    for i, (pa, pb) in enumerate(zip(a["params"], b["params"])):
        assert np.array_equal(pa, pb), f"step {i}: ranks' parameters differ"
    assert not np.array_equal(a["params"][0], a["params"][-1])        # training moved them
    for ta, tb in zip(a["targets"], b["targets"]):
        assert not np.array_equal(ta, tb)                               # different batches
    assert all(np.isfinite(x["loss"]).all() for x in (a, b))


def _union_worker(rank, world, port, q):
    """rank r of 2 trains the fused step on half r of a fixed 64-target batch (the same hop seed
    as the union: samples are keyed on (hop seed, node)), all-reduces the flat gradient bucket and
    takes FlatAdam's step with grad_scale = 1/2 (what bench.py runs at world > 1); rank 0 then runs
    one world-1 step on the union (Adam inside the step's last launch)."""
    try:
        import torch.distributed as dist
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        sys.path.insert(0, HERE)
        sys.path.insert(0, os.path.join(os.path.dirname(HERE), "re-gnn_amd"))
        from test_gpu_ns_engine import _mag
        from regnn_hip import ns
        from regnn_hip.ns import NSTrainer
        ns.SPLIT_EXCHANGE["mode"] = "on"       # the split exchange's gradients under the contract
        d = _mag(0.002, seed=8, F=128, hidden=64, classes=13, dropout=0.0)
        union = torch.randperm(d["n_paper"], generator=torch.Generator().manual_seed(0))[:64]
        union = union.to("cuda")

        def trainer(w, r):
            return NSTrainer(d["model"](5), None, d["rg"], [6, 4], 64,
                             torch.arange(d["n_paper"], device="cuda"), d["x_dict"],
                             d["edge_type"], d["node_type"], d["local"], d["y"], 7, seed=9,
                             rank=r, world=w, adam=dict(lr=1e-2), pipeline=False)

        def one_step(tr, targets):
            s = tr.slots[0]
            s.set_seed(11, 0, 4)
            s.set_targets(targets)
            s.run_hops()
            tr._fs_step(tr.fused)              # (several ranks: the split exchange's first part)
            tr._exchange()
            tr._opt_step()
            torch.cuda.synchronize()

        tr = trainer(world, rank)
        assert tr.fused is not None and tr.fused.two_layer and not tr.adam_fused
        assert tr._xsplit and 0 < tr.n_early < tr.flat.numel()
        assert tr.opt.grad_scale == 0.5
        one_step(tr, union[32 * rank:32 * (rank + 1)])
        out = {"grad_sum": tr.flat.cpu().numpy().copy(),
               "param": tr.param_vector().cpu().numpy().copy()}
        dist.barrier()
        dist.destroy_process_group()
        if rank == 0:
            tu = trainer(1, 0)
            assert tu.adam_fused
            one_step(tu, union)
            out["union_grad"] = tu.flat.cpu().numpy().copy()
            out["layout"] = [(o, p.numel()) for o, p in zip(tu.offsets, tu.params)]
            out["union_param"] = tu.param_vector().cpu().numpy().copy()
            out["param0"] = torch.cat([p.detach().reshape(-1) for p in
                                       d["model"](5).parameters()]).cpu().numpy()
        q.put((rank, out))
    except Exception as e:                      # surface the failure in the parent
        import traceback
        q.put((rank, repr(e) + traceback.format_exc()))


def test_ns_dp_fused_union_equals_allreduced_halves():
    """the data-parallel contract of the fused step the bench runs. Two ranks
    (gloo, one GPU) each run regnn_nsm_step on half of a batch; the SUM all-reduce plus FlatAdam's
    grad_scale = 1/2 give the gradient and the Adam update of one world-1 step on the union batch
    (mag/regnn_ns.py:405-407 under DistributedDataParallel)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + ((os.getpid() + 500) % 1000)
    procs = [ctx.Process(target=_union_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for r in (0, 1):
        assert not isinstance(res[r], str), f"rank {r}: {res[r]}"
    a, b = res[0], res[1]
    assert np.array_equal(a["grad_sum"], b["grad_sum"])
    assert np.array_equal(a["param"], b["param"])
    g_dp = 0.5 * a["grad_sum"].astype(np.float64)          # padded buckets, same layout
    g_u = a["union_grad"].astype(np.float64)
    scale = max(1e-3, float(np.abs(g_u).max()))
    assert np.abs(g_dp - g_u).max() <= 2e-6 * scale, np.abs(g_dp - g_u).max()
    # Adam's first step moves each element by lr * g / (|g| + eps): equal wherever the gradient
    # is not within rounding of zero
    moved = np.abs(a["union_param"] - a["param0"])
    assert moved.max() > 1e-3
    d = np.abs(a["param"].astype(np.float64) - a["union_param"])
    g_uv = np.concatenate([g_u[o:o + n] for o, n in a["layout"]])
    sure = np.abs(g_uv) > 1e-4 * scale
    assert d[sure].max() <= 1e-6, d[sure].max()
    assert d.max() <= 2.01e-2


def _graph_allreduce_worker(port, q):
    try:
        import torch.distributed as dist
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=0, world_size=1)
        sys.path.insert(0, HERE)
        sys.path.insert(0, os.path.join(os.path.dirname(HERE), "re-gnn_amd"))
        from test_gpu_ns_engine import _mag
        from regnn_hip.ns import NSTrainer
        d = _mag(0.002, seed=8, F=128, hidden=64, classes=13, dropout=0.3)

        def make():
            return NSTrainer(d["model"](5), None, d["rg"], [6, 4], 64,
                             torch.arange(d["n_paper"], device="cuda"), d["x_dict"],
                             d["edge_type"], d["node_type"], d["local"], d["y"], 7, seed=9,
                             adam=dict(lr=1e-2))
        from regnn_hip import ns
        ta, tb, tc = make(), make(), make()
        ta._force_exchange = True              # the RCCL all-reduce inside the captured graph
        ta.capture(warmup=1, exchange_in_graph=True)
        tb.capture(warmup=1)
        # the several-rank structure: split finalize, the early all-reduce on the comm stream
        # between the step's parts, the rest after it, Adam as its own launch (regnn_adam_flat:
        # equal to the fused Adam within rounding, test_fused_adam_equals_separate_adam)
        ns.SPLIT_EXCHANGE["mode"] = "on"
        tc.rehearse_exchange()
        assert tc._xsplit and not tc.adam_fused
        tc.capture(warmup=1, exchange_in_graph=True)
        assert ta.graphs[1] is None and ta.graph_groups and tc.graph_groups
        out = []
        for k in (4, 1, 3):                    # a multi-step graph first, then single replays
            for t in (ta, tb, tc):
                t.run_steps(k)
            torch.cuda.synchronize()
            out.append((float(ta.loss), float(tb.loss), bool(torch.equal(ta.pflat, tb.pflat)),
                        abs(float(tc.loss) - float(tb.loss)) <= 1e-5 * abs(float(tb.loss)) and
                        bool(torch.allclose(tc.pflat, tb.pflat, rtol=1e-5, atol=1e-6))))
        dist.destroy_process_group()
        q.put(out)
    except Exception as e:
        import traceback
        q.put(repr(e) + traceback.format_exc())


def test_ns_allreduce_captured_in_step_graph():
    """NSTrainer.capture(exchange_in_graph=True): the flat-bucket RCCL all-reduce captured inside
    the step's HIP graph (one replay per step, runs of steps as one replay) on a one-rank NCCL
    group; it must replay and train exactly as the one-rank graph without the exchange."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + ((os.getpid() + 250) % 1000)
    p = ctx.Process(target=_graph_allreduce_worker, args=(port, q))
    p.start()
    res = q.get(timeout=150)
    p.join(timeout=60)
    assert not isinstance(res, str), res
    for la, lb, same, same_split in res:
        assert la == lb and same and same_split


def _fallback_worker(rank, world, port, q):
    """rank 1's in-graph capture fails (injected), rank 0's succeeds (its captured exchange
    stubbed: gloo cannot be captured): capture() must agree across ranks and fall back to the
    eager exchange on BOTH, with the fallback really capturing without the exchange."""
    try:
        import torch.distributed as dist
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        sys.path.insert(0, HERE)
        sys.path.insert(0, os.path.join(os.path.dirname(HERE), "re-gnn_amd"))
        import warnings
        from test_gpu_ns_engine import _mag
        from regnn_hip.ns import NSTrainer
        d = _mag(0.002, seed=8, F=128, hidden=64, classes=13, dropout=0.3)

        def make():
            return NSTrainer(d["model"](5), None, d["rg"], [6, 4], 64,
                             torch.arange(d["n_paper"], device="cuda"), d["x_dict"],
                             d["edge_type"], d["node_type"], d["local"], d["y"], 7, seed=9,
                             rank=rank, world=world, adam=dict(lr=1e-2))

        out = {}
        for mode in ("fallback", "eager"):
            tr = make()
            if mode == "fallback":
                def stub(orig):
                    def exchange():
                        if torch.cuda.is_current_stream_capturing():
                            if rank == 1:
                                raise RuntimeError("injected: all-reduce capture failed")
                            return              # rank 0: a captured collective's stand-in
                        orig()
                    return exchange
                # (the split exchange's early all-reduce too: the first collective of a step)
                tr._exchange = stub(tr._exchange)
                tr._exchange_early = stub(tr._exchange_early)
                with warnings.catch_warnings(record=True) as wl:
                    warnings.simplefilter("always")
                    tr.capture(warmup=1, exchange_in_graph=True)
                out["warned"] = any("falls back" in str(w.message) for w in wl)
            else:
                tr.capture(warmup=1, exchange_in_graph=False)
            out[mode + "_in_graph"] = tr.exchange_in_graph
            out[mode + "_g2"] = tr.graphs[1] is not None
            losses = []
            for k in (3, 1, 2):
                tr.run_steps(k)
                torch.cuda.synchronize()
                losses.append(float(tr.loss))
            tr.step()                           # and an eager step after the replays
            torch.cuda.synchronize()
            out[mode] = tr.pflat.detach().cpu().numpy().copy()
            out[mode + "_loss"] = losses
            dist.barrier()
        dist.destroy_process_group()
        q.put((rank, out))
    except Exception as e:
        import traceback
        q.put((rank, repr(e) + traceback.format_exc()))


def test_capture_fallback_agreed_across_ranks():
    """VERDICT r3 next 1 (a, b): capture(exchange_in_graph=True) failing on one rank only makes
    every rank fall back to the eager exchange (a MAX all-reduce of the failure flags before any
    replay), the fallback captures without the exchange, and both ranks then train bitwise the
    same parameters as a run that chose the eager exchange from the start."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + ((os.getpid() + 750) % 1000)
    procs = [ctx.Process(target=_fallback_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for r in (0, 1):
        assert not isinstance(res[r], str), f"rank {r}: {res[r]}"
    a, b = res[0], res[1]
    for x in (a, b):
        assert x["warned"]
        assert not x["fallback_in_graph"] and x["fallback_g2"]
        assert not x["eager_in_graph"] and x["eager_g2"]
        assert np.array_equal(x["fallback"], x["eager"])
        assert x["fallback_loss"] == x["eager_loss"]
    assert np.array_equal(a["fallback"], b["fallback"])
    assert np.isfinite(a["eager_loss"]).all()


def test_bench_self_launch_two_ranks():
    """`python bench.py --gpus 2` with no launcher environment starts the
    two ranks itself (gloo on the box's one GPU) and prints one JSON line with n_gpus 2."""
    import json
    import subprocess
    root = os.path.dirname(HERE)
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["REGNN_DIST_BACKEND"] = "gloo"
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2",
                        "--scale", "0.2", "--steps", "4", "--warmup", "2"],
                       cwd=root, env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["config"]["parallelism"] == "dp2"
    assert rec["config"]["grad_exchange"] == "eager all-reduce between graphs"
    assert rec["value"] > 0
