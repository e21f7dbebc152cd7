"""world_size-2 gloo rehearsal of bench.py's own multi-rank plumbing (CPU):
process-group init from the torch.distributed.run environment, the
configs[4] strong-scaling slab split (fa_hip.shard.shard_range), the barrier +
MAX-over-ranks timing reduction and the JSON block — the code the driver's
8-GPU run executes with RCCL, here with gloo and a CPU step supplied by the
test (the product step is the HIP kernel; bench.py never computes on the CPU)."""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

import bench


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      LOCAL_RANK=str(rank), WORLD_SIZE=str(world))
    dist, r, w, _ = bench.dist_init("gloo")
    assert (r, w) == (rank, world) and dist is not None
    try:
        from oracle import fa_oracle as O
        N, d, total = 32, 8, 7
        rng = np.random.default_rng(5)
        q, k, v = (rng.standard_normal((N, d, total)) for _ in range(3))
        from fa_hip.shard import shard_range
        seen = {}

        def make_step(n_local):
            a, b = shard_range(total, w, r)
            assert b - a == n_local
            seen["n"] = n_local

            def step():
                y, _, _ = O.dense_fa3(q[..., a:b], k[..., a:b], v[..., a:b])
                seen["y"] = y
                if r == 1:
                    time.sleep(0.05)        # the slow rank sets the reported time
            return step

        res = bench.sharded_strong(make_step, total, w, r, dist, steps=2, warmup=1,
                                   flops_per_slab=4.0 * N * N * d, sync=lambda: None, events=False)
        json.dumps(res)
        a, b = shard_range(total, w, r)
        ref, _, _ = O.dense_fa3(q, k, v)
        out[rank] = dict(res=res, err=float(np.abs(seen["y"] - ref[..., a:b]).max()))
    finally:
        dist.barrier()
        dist.destroy_process_group()


def test_bench_strong_scaling_plumbing_two_ranks():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    assert sorted(out.keys()) == [0, 1]
    r0, r1 = out[0]["res"], out[1]["res"]
    assert r0["slab_split"] == [[0, 4], [4, 7]] == r1["slab_split"]
    assert (r0["slabs_this_rank"], r1["slabs_this_rank"]) == (4, 3)
    # MAX over ranks: both ranks report the slow rank's time (>= its 50 ms sleep)
    assert r0["ms_per_step_max_over_ranks"] == r1["ms_per_step_max_over_ranks"] >= 50.0
    assert r0["tflops_total"] == r1["tflops_total"]
    assert abs(r0["tflops_per_gpu"] * 2 - r0["tflops_total"]) < 1e-12
    assert r0["scaling"] == "strong" and r0["n_gpus"] == 2
    assert max(out[0]["err"], out[1]["err"]) < 1e-12


def test_cpu_threads_respects_share(monkeypatch):
    monkeypatch.setenv("OMP_NUM_THREADS", "3")
    assert bench._cpu_threads() == min(3, len(os.sched_getaffinity(0)))
    assert bench._node_cpus() == len(os.sched_getaffinity(0))     # the node legs ignore the share
    monkeypatch.delenv("OMP_NUM_THREADS")
    assert bench._cpu_threads() == len(os.sched_getaffinity(0))


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench_env(**extra):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    env.update(FA_BENCH_CPU_STEP="1", FA_BENCH_BACKEND="gloo", OMP_NUM_THREADS="1", **extra)
    return env


# the CPU step hook (FA_BENCH_CPU_STEP) is refused where a GPU is visible
_cpu_only = pytest.mark.skipif(torch.cuda.is_available(), reason="CPU step hook: refused on a GPU box")


@_cpu_only
def test_bench_gpus_2_literal_command_spawns_two_ranks():
    """The driver's literal form `python bench.py --gpus 2` (no torch.distributed.run
    around it) starts two ranks itself; with the CPU step hook (rank r sleeps
    (r + 1) * 5 ms per step) the JSON line must say n_gpus 2, split configs[4]'s 1024
    slabs as [[0, 512], [512, 1024]] and report the MAX over ranks (the slow rank)."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "4",
                        "--warmup", "1", "--cfg4-steps", "2", "--no-cpu"],
                       cwd=ROOT, env=_bench_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout          # rank 0 only
    out = json.loads(lines[0])
    assert out["cpu_step_hook"] is True
    assert out["n_gpus"] == 2 and out["config"]["global_batch_heads"] == 128
    assert out["config"]["parallelism"].startswith("shard(B*H) x2")
    # MAX over ranks: rank 1's 10 ms per step, not rank 0's 5 ms
    assert out["ms_per_step"] >= 10.0
    c4 = out["cfg4"]
    assert c4["n_gpus"] == 2 and c4["slab_split"] == [[0, 512], [512, 1024]]
    assert c4["slabs_this_rank"] == 512 and c4["ms_per_step_max_over_ranks"] >= 10.0
    assert abs(c4["tflops_per_gpu"] * 2 - c4["tflops_total"]) < 1e-9 * c4["tflops_total"]
    # aggregate over both ranks: value = world * per-rank FLOPs / the slowest rank's time
    flops_rank = 4.0 * 64 * 4096 * 4096 * 64
    assert abs(out["value"] - 2 * flops_rank * 4 / (out["ms_per_step"] * 4 / 1e3) / 1e12) < 1e-6 * out["value"]


@_cpu_only
def test_bench_refuses_gpus_world_mismatch():
    """Under torch.distributed.run, --gpus must equal WORLD_SIZE (exit 2), and
    --gpus < 1 is refused, before anything is measured."""
    env = _bench_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "WORLD_SIZE=1" in r.stderr
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "0"],
                       cwd=ROOT, env=_bench_env(), capture_output=True, text=True, timeout=120)
    assert r.returncode == 2


def test_cpu_baseline_legs_small(monkeypatch):
    """cpu_baseline's legs on a reduced workload (CPU): the BLAS port and the plain
    OpenMP port agree with each other, and the node legs cap the BLAS callers at
    numpy's OpenBLAS limit."""
    import numpy as np
    monkeypatch.setattr(bench, "N_", 256)
    monkeypatch.setattr(bench, "B_", 1)
    monkeypatch.setattr(bench, "H_", 2)
    monkeypatch.setattr(bench, "_node_cpus", lambda: 2)
    monkeypatch.setenv("OMP_NUM_THREADS", "1")
    out = bench.cpu_baseline(node=True)
    assert set(out["legs"]) == {"share", "node_blas", "node_plain"}
    assert out["legs"]["node_blas"]["threads"] == min(2, bench.OPENBLAS_MAX_CALLERS)
    assert out["value"] > 0 and out["cores"] in (1, 2)
    from oracle import cpu_port
    rng = np.random.default_rng(1)
    q, k, v = (np.asfortranarray(rng.standard_normal((96, 16, 2)).astype(np.float32)) for _ in range(3))
    a = cpu_port.dense_fa_blas(q, k, v, 2)[0]
    b = bench._plain_port(q, k, v, 2)
    assert np.abs(a - b).max() < 1e-5
