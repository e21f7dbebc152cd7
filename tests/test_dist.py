"""world_size-2 gloo tests of the (batch × head) sharding used by bench.py and
fa_hip.shard (CPU only; the per-slab compute is the CPU oracle here, the GPU
path is the same call on a device slab)."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from fa_hip.shard import gather_slabs, local_slabs, shard_range


def test_shard_range_partitions():
    for n in (1, 7, 64, 1024):
        for w in (1, 2, 3, 8):
            got = [shard_range(n, w, r) for r in range(w)]
            assert got[0][0] == 0 and got[-1][1] == n
            assert all(got[i][1] == got[i + 1][0] for i in range(w - 1))
            sizes = [b - a for a, b in got]
            assert max(sizes) - min(sizes) <= 1


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
    try:
        from oracle import fa_oracle as O
        rng = np.random.default_rng(0)                 # identical global inputs on every rank
        N, d, BH = 48, 16, 5
        q, k, v = (rng.standard_normal((N, d, BH)) for _ in range(3))
        jl = lambda a: torch.tensor(a).permute(2, 1, 0).contiguous().permute(2, 1, 0)
        Q, K, V = jl(q), jl(k), jl(v)
        lq, lk, lv = (local_slabs(t, world, rank) for t in (Q, K, V))
        a, b = shard_range(BH, world, rank)
        # a zero-copy view: the rank's slabs are one contiguous byte range of the global array
        assert lq.data_ptr() == Q.data_ptr() + a * N * d * Q.element_size()
        assert lq.shape == (N, d, b - a) and lq.stride() == Q.stride()
        y, l, m = O.dense_fa3(lq.numpy(), lk.numpy(), lv.numpy())   # per-rank compute, no collective
        yl = jl(y)
        full = gather_slabs(yl, BH)
        ref, _, _ = O.dense_fa3(q, k, v)
        out[rank] = float(np.abs(full.numpy() - ref).max())
        # the timing reduction bench.py uses (MAX over ranks)
        t = torch.tensor([float(rank + 1)])
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        assert float(t[0]) == world
    finally:
        dist.destroy_process_group()


def test_two_rank_sharded_dense_matches_full():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    assert len(out) == world and max(out.values()) < 1e-12
