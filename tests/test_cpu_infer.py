"""Host logic of the sharded full-neighbour inference (regnn_hip/inference.py, SURVEY.md §8f
rank 1): row sharding, the per-rank row block (CSR row range + appended self loops, as
mag/regnn_layers.py:90-96 builds them) and the all-gather exchange on world_size 2 (gloo)."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from regnn_hip.graph import RelGraph
from regnn_hip.inference import RowBlock, exchange_rows, shard_bounds


def _powerlaw_graph(n=3000, m=40000, seed=0):
    rng = np.random.default_rng(seed)
    dst = (rng.zipf(1.3, m) - 1) % n
    src = rng.integers(0, n, m)
    et = rng.integers(0, 7, m)
    ntype = rng.integers(0, 4, n)
    return src, dst, et, ntype, n


def test_shard_bounds_cover_and_balance():
    src, dst, et, ntype, n = _powerlaw_graph()
    rg = RelGraph(src, dst, n, "cpu")
    for world in (1, 2, 3, 8):
        b = shard_bounds(rg.csr_ptr, world)
        assert b[0] == 0 and b[-1] == n and len(b) == world + 1
        assert all(b[i] <= b[i + 1] for i in range(world))
        ptr = rg.csr_ptr.to(torch.int64)
        cost = [int(ptr[b[r + 1]] - ptr[b[r]]) + b[r + 1] - b[r] for r in range(world)]
        total = src.size + n
        heaviest_row = int((ptr[1:] - ptr[:-1]).max()) + 1
        assert max(cost) <= total / world + heaviest_row


def test_row_block_matches_reference_block():
    src, dst, et, ntype, n = _powerlaw_graph(seed=1)
    rg = RelGraph(src, dst, n, "cpu")
    et_csr = torch.from_numpy(et)[rg.csr_eid].to(torch.uint8)
    nt = torch.from_numpy(ntype)
    for r0, r1 in ((0, n), (17, 950), (n - 5, n)):
        blk = RowBlock(rg, r0, r1, et_csr, nt, 7)
        ptr = blk.csr_ptr.numpy()
        idx = blk.csr_idx.numpy()
        rel = blk.pack.rel_csr.numpy()
        assert blk.n_dst == r1 - r0 and blk.n_src == n and blk.E == ptr[-1]
        for i in range(r1 - r0):
            v = r0 + i
            a, b = ptr[i], ptr[i + 1]
            # self loop last, typed ntype + num_edge_types (mag/regnn_layers.py:90-96)
            assert idx[b - 1] == v and rel[b - 1] == ntype[v] + 7
            want = np.nonzero(dst == v)[0]                 # in-edges in edge-id order
            assert np.array_equal(idx[a:b - 1], src[want])
            assert np.array_equal(rel[a:b - 1], et[want])
        cnt = np.bincount(dst, minlength=n)[r0:r1] + 1
        assert np.allclose(blk.inv_in_count().numpy(), 1.0 / cnt)


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
    bounds = [0, 7, 19] if world == 2 else None                  # uneven shards
    full = torch.arange(19 * 5, dtype=torch.float32).view(19, 5)
    mine = full[bounds[rank]:bounds[rank + 1]].clone()
    got = exchange_rows(mine, bounds, rank, world)
    out[rank] = bool(torch.equal(got, full))
    dist.destroy_process_group()


def test_exchange_rows_two_ranks():
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    assert out[0] and out[1]
