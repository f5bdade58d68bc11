"""The data-parallel NS step with two ranks on the box's one GPU (gloo standing in for RCCL, which
cannot run two ranks on one device): the pipelined two-slot trainer with world = 2 captured as
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
