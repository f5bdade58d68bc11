"""Multi-process (world_size 2, gloo, CPU) checks of the data-parallel machinery of the
neighbour-sampled path: batch dealing across ranks and the flat-bucket gradient all-reduce
(regnn_hip.mag.flat_grad_allreduce, mag/regnn_ns.py:406-407)."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


class _StubGraph:
    def __init__(self, n):
        self.n_dst, self.device = n, torch.device("cpu")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from regnn_hip.mag import flat_grad_allreduce
    from regnn_hip.sampler import NeighborSampler
    # 1. batch dealing: shared permutation, rank r takes global batches r, r+W, ...
    smp = NeighborSampler(_StubGraph(1000), torch.arange(1000), [25, 20], batch_size=64,
                          shuffle=True, seed=5, rank=rank, world_size=world)
    smp.set_epoch(2)
    mine = [(b, t.tolist()) for b, t in smp.batches()]
    # 2. gradient all-reduce: each rank the mean loss of its half of a global batch
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.ReLU(), torch.nn.Linear(16, 3))
    g = torch.Generator().manual_seed(1)
    X = torch.randn(64, 8, generator=g)
    Y = torch.randint(0, 3, (64,), generator=g)
    part = slice(rank * 32, (rank + 1) * 32)
    loss = torch.nn.functional.cross_entropy(model(X[part]), Y[part])
    loss.backward()
    flat_grad_allreduce(list(model.parameters()), world)
    out[rank] = {"batches": mine, "grads": [p.grad.clone() for p in model.parameters()]}
    dist.destroy_process_group()


def test_dp_two_ranks():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    b0, b1 = out[0]["batches"], out[1]["batches"]
    assert all(b % 2 == 0 for b, _ in b0) and all(b % 2 == 1 for b, _ in b1)
    nodes = [x for _, t in b0 + b1 for x in t]
    assert sorted(nodes) == list(range(1000))            # disjoint cover of the train nodes
    # single-process reference: mean loss over the whole global batch
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.ReLU(), torch.nn.Linear(16, 3))
    g = torch.Generator().manual_seed(1)
    X = torch.randn(64, 8, generator=g)
    Y = torch.randint(0, 3, (64,), generator=g)
    torch.nn.functional.cross_entropy(model(X), Y).backward()
    for r in range(world):
        for got, p in zip(out[r]["grads"], model.parameters()):
            assert torch.allclose(got, p.grad, atol=1e-6, rtol=1e-5)


def _sparse_worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from regnn_hip.mag import sparse_rows_allreduce
    g = torch.Generator().manual_seed(10 + rank)
    table = torch.nn.Parameter(torch.zeros(50, 6))
    rows = torch.tensor([[1, 4, 7, 9, 30], [4, 5, 9, 49]][rank])        # overlapping rows
    table.grad = torch.zeros(50, 6)
    table.grad[rows] = torch.randn(rows.numel(), 6, generator=g)
    dense = table.grad.clone()
    dist.all_reduce(dense)
    dense /= world
    sparse_rows_allreduce([(table, rows)], world)
    out[rank] = (table.grad.clone(), dense)
    dist.destroy_process_group()


def test_sparse_rows_allreduce_two_ranks():
    """feats_type-2 embedding tables: the touched-rows exchange gives the
    dense SUM / world all-reduce on every rank, identically."""
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_sparse_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    (g0, d0), (g1, d1) = out[0], out[1]
    assert torch.equal(g0, g1)
    assert torch.allclose(g0, d0, atol=1e-6) and torch.allclose(g1, d1, atol=1e-6)


def _uneven_worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from regnn_hip.mag import flat_grad_allreduce
    from regnn_hip.sampler import NeighborSampler
    # 1000 targets / batch 200 = 5 global batches over 2 ranks: rank 1 wraps to batch 0, so both
    # ranks run 3 steps and every per-step all-reduce has its partner (no hang at epoch end)
    smp = NeighborSampler(_StubGraph(1000), torch.arange(1000), [25, 20], batch_size=200,
                          shuffle=True, seed=9, rank=rank, world_size=world)
    model = torch.nn.Linear(4, 2)
    steps = []
    for b, t in smp.batches():
        model.zero_grad()
        model(t.float().reshape(-1, 1).repeat(1, 4)[:8] / 1000).sum().backward()
        flat_grad_allreduce(list(model.parameters()), world)
        steps.append(b)
    out[rank] = steps
    dist.destroy_process_group()


def test_dp_uneven_batch_count_same_steps_per_rank():
    """nb % world != 0 must not leave one rank alone in the gradient all-reduce."""
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_uneven_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    assert out[0] == [0, 2, 4] and out[1] == [1, 3, 0]


_FAIL_WORKER = r"""
import os, sys, time
sys.path.insert(0, os.path.join(os.environ["REGNN_ROOT"], "re-gnn_amd"))
import torch
import torch.distributed as dist
from regnn_hip.guard import Guard, pg_timeout
from regnn_hip.ns import NSTrainer

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dist.init_process_group("gloo", rank=rank, world_size=world, timeout=pg_timeout())


class FakeTrainer:
    # NSTrainer.guarded_step's contract on the CPU: forward / backward local, the exchange a
    # collective every rank issues, then the optimizer
    world = 2

    def __init__(self):
        self.flat = torch.ones(1000)
        self.steps = 0

    def _forward_backward(self):
        self.flat.mul_(1.5)
        if rank == 1 and self.steps == int(os.environ["FAIL_AT"]):
            if os.environ.get("FAIL_MODE") == "die":
                os._exit(9)                              # a hard death: no agreement from it
            raise RuntimeError("injected failure inside the warm-up step")

    def _exchange(self):
        dist.all_reduce(self.flat)

    def _opt_step(self):
        self.steps += 1


tr = FakeTrainer()
guard = Guard(world)
guard.stage("build", lambda: None)
for _ in range(3):                                   # the warm-up steps
    NSTrainer.guarded_step(tr, guard)
print(f"rank {rank} finished", flush=True)
dist.destroy_process_group()
"""


def _run_two_ranks(fail_at, timeout_s=20, mode="raise"):
    import subprocess
    import sys
    import time
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    port = _free_port()
    procs = []
    t0 = time.time()
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), REGNN_ROOT=root, FAIL_AT=str(fail_at), FAIL_MODE=mode,
                   REGNN_DIST_TIMEOUT=str(timeout_s))
        procs.append(subprocess.Popen([sys.executable, "-c", _FAIL_WORKER], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = []
    for p in procs:
        try:
            o, e = p.communicate(timeout=timeout_s + 60)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise AssertionError("a rank hung past the process group timeout")
        outs.append((p.returncode, o, e))
    return outs, time.time() - t0


def test_rank_failure_in_warmup_ends_every_rank():
    """rank 1 raises inside a warm-up step (its peer is then in the step's
    gradient all-reduce); both ranks exit non-zero (guard.EXIT_CODE) well within the process
    group's timeout, neither hangs, and rank 1 reports the injected error."""
    from regnn_hip.guard import EXIT_CODE
    outs, dt = _run_two_ranks(fail_at=1)
    codes = [rc for rc, _, _ in outs]
    assert codes == [EXIT_CODE, EXIT_CODE], (codes, [e[-600:] for _, _, e in outs])
    assert "injected failure" in outs[1][2]
    assert all("finished" not in o for _, o, _ in outs)
    assert dt < 20, dt                                 # agreement, not the timeout, ended it


def test_peer_death_ends_the_survivor_with_exit_code():
    """rank 1 dies without reaching the agreement (os._exit inside the step); rank 0's
    exchange and then its agreement all-reduce fail, and the guarded agreement turns that into
    RankFailure: rank 0 exits guard.EXIT_CODE (not a plain RuntimeError traceback), in time."""
    from regnn_hip.guard import EXIT_CODE
    outs, dt = _run_two_ranks(fail_at=1, mode="die")
    codes = [rc for rc, _, _ in outs]
    assert codes == [EXIT_CODE, 9], (codes, [e[-600:] for _, _, e in outs])
    assert "finished" not in outs[0][1]
    assert dt < 60, dt


def test_no_failure_both_ranks_finish():
    outs, _ = _run_two_ranks(fail_at=-1)
    assert [rc for rc, _, _ in outs] == [0, 0], [e[-600:] for _, _, e in outs]
    assert all("finished" in o for _, o, _ in outs)
