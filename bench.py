"""bench.py — headline benchmark (BASELINE.json metric).

metric : effective attention TFLOP/s (fwd) at N=4096, d=64; % of bf16 MFMA peak
step   : one fa_dense_fwd call over this rank's (B·H) slabs of BASELINE
         configs[1] = (B,H,N,d) = (4,16,4096,64) bf16, i.e. (N, d, B·H) =
         (4096, 64, 64) in the reference's column-major layout; inputs resident
         in HBM before the timed region.
FLOPs  : 4·(B·H)·N²·d per step per rank (non-causal; softmax not counted;
         SURVEY.md §8d).
scaling: weak — every rank processes its own 64 slabs (sharding over
         batch × head, no data-path collective; a gloo/RCCL barrier and a MAX
         all-reduce of the elapsed time are the only cross-rank calls).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu] [--extra]
Multi-GPU: python -m torch.distributed.run --nnodes=1 --nproc-per-node N
           --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "flashattention.jl_amd")
for _p in (ROOT, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402

METRIC = "effective attention TFLOP/s (fwd) at N=4096,d=64; % of bf16 MFMA peak"
PEAK_BF16_TFLOPS = 256 * 2.4e9 * 4096 / 1e12   # 2516.6: 256 CU x 2.4 GHz x 4096 FLOP/clk/CU (dense)
PEAK_HBM_GBS = 8000.0
B_, H_, N_, D_ = 4, 16, 4096, 64


def _dist_init(n_gpus):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        return dist, rank, world, local
    torch.cuda.set_device(0)
    return None, 0, 1, 0


def _randn_jl(fa, shape, dtype, gen):
    t = fa.jl_empty(shape, dtype)
    t.copy_(torch.randn(tuple(shape), generator=gen, device="cuda", dtype=torch.float32))
    return t


def time_launches(fn, steps, warmup, dist=None):
    """Barrier + sync on both sides; returns (max-over-ranks wall s, event s)."""
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(steps):
        fn()
    ev1.record(stream)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    wall = time.perf_counter() - t0
    ev_s = ev0.elapsed_time(ev1) / 1e3
    if dist is not None:
        t = torch.tensor([wall, ev_s], device="cuda", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall, ev_s = float(t[0]), float(t[1])
    return wall, ev_s


def time_graph(fn, steps, dist=None):
    """Device time per call of a launch-bound fn: `steps` calls captured in one
    HIP graph (torch.cuda.graph) and replayed, so host issue overhead (Python +
    ctypes, ~20-30 us per call) is not what gets measured for kernels of a few
    microseconds.  Barrier + sync on both sides, max over ranks."""
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(2):
            fn()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        for _ in range(steps):
            fn()
    graph.replay()
    torch.cuda.synchronize()
    _, e = time_launches(graph.replay, 3, 1, dist)
    return e / 3 / steps


def cpu_baseline(target_s: float = 12.0):
    """oracle/fa_cpu.c (C OpenMP port of dense_fa!, src/dense.jl:21-102, same
    Br=64/Bc=500 tiles) on a bounded sample of the same workload: whole
    (4096, 64) slabs in fp32, as many as fit ~target_s of CPU time."""
    import numpy as np
    from oracle import cpu_port
    threads = min(16, os.cpu_count() or 1)
    rng = np.random.default_rng(0)
    one = lambda n: [np.asfortranarray(rng.standard_normal((N_, D_, n)).astype(np.float32)) for _ in range(3)]
    q, k, v = one(1)
    cpu_port.dense_fa(q, k, v, threads)              # warm-up
    t = time.perf_counter()
    cpu_port.dense_fa(q, k, v, threads)
    per_slab = time.perf_counter() - t
    n = int(max(1, min(64, target_s / max(per_slab, 1e-6))))
    q, k, v = one(n)
    reps, dts = max(1, min(5, int(target_s / max(per_slab * n, 1e-6)))), []
    for _ in range(reps):                              # best of a few full passes
        t = time.perf_counter()
        cpu_port.dense_fa(q, k, v, threads)
        dts.append(time.perf_counter() - t)
    dt = min(dts)
    flops = 4.0 * n * N_ * N_ * D_
    return {"value": flops / dt / 1e12, "unit": "TFLOP/s", "cores": threads, "kind": "port",
            "sample": f"{n} of 64 (N,d)=(4096,64) slabs of configs[1], fp32, C/OpenMP port of dense_fa! "
                      f"(oracle/fa_cpu.c, reference tiles Br=64 Bc=500), best of {reps}: {dt:.2f} s"}


def _traffic_from_profiles():
    """HBM bytes per launch of the forward kernel from the committed rocprofv3
    PMC summary (profiles/*fwd_traffic*.json, written by
    profiles/pmc_traffic.py from separate FETCH_SIZE / WRITE_SIZE passes with
    the gfx950 FETCH_SIZE x2 correction), if one exists for this workload."""
    import glob
    best = None
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "*fwd_traffic*.json"))):
        try:
            j = json.load(open(p))
        except Exception:
            continue
        if j.get("workload") == "configs[1]":
            best = j.get("hbm_bytes_per_launch")
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    # ~0.1 s of untimed launches: from idle the GPU needs ~200 launches (~60 ms)
    # to reach its sustained clock (tools/exp/ramp.py)
    ap.add_argument("--warmup", type=int, default=400)
    ap.add_argument("--no-cpu", action="store_true", help="skip the cpu_baseline leg")
    ap.add_argument("--extra", action="store_true", help="also time configs[2..3] (reported under 'extra')")
    args = ap.parse_args()

    dist, rank, world, local = _dist_init(args.gpus)
    import fa_hip
    fa_hip.lib()

    BH = B_ * H_
    gen = torch.Generator(device="cuda").manual_seed(1234 + rank)
    Q = _randn_jl(fa_hip, (N_, D_, BH), torch.bfloat16, gen)
    K = _randn_jl(fa_hip, (N_, D_, BH), torch.bfloat16, gen)
    V = _randn_jl(fa_hip, (N_, D_, BH), torch.bfloat16, gen)
    O = fa_hip.jl_empty((N_, D_, BH), torch.bfloat16)
    l = fa_hip.jl_empty((N_, 1, BH), torch.float32)
    m = fa_hip.jl_empty((N_, 1, BH), torch.float32)
    step = lambda: fa_hip.dense_fa_(O, l, m, Q, K, V)

    wall, ev_s = time_launches(step, args.steps, args.warmup, dist)
    flops_rank = 4.0 * BH * N_ * N_ * D_
    value = flops_rank * world * args.steps / wall / 1e12
    kern_s = ev_s / args.steps
    achieved = flops_rank / kern_s / 1e12

    out = {
        "metric": METRIC, "value": value, "unit": "TFLOP/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": wall / args.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
        "data": "synthetic (torch.randn -> bf16, column-major (N,d,B*H) device arrays)",
        "config": {"workload": "configs[1]: dense_fa bf16 forward, (B,H,N,d)=(4,16,4096,64) per GPU",
                   "B": B_, "H": H_, "N": N_, "d": D_, "slabs_per_gpu": BH,
                   "global_batch_heads": BH * world, "parallelism": f"shard(B*H) x{world}, no collective"},
        "roofline": {"bound": "mfma", "achieved": achieved, "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                     "frac": achieved / PEAK_BF16_TFLOPS, "traffic": _traffic_from_profiles(),
                     "kernel": "fa::dense_fwd_w8q2<bf16,64,64>",
                     "flops_per_launch": flops_rank, "avg_launch_ms": kern_s * 1e3},
    }

    if args.extra:
        out["extra"] = extra_benches(fa_hip, args, dist)

    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline()
    elif rank == 0:
        out["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def extra_benches(fa_hip, args, dist):
    """Secondary BASELINE configs (not the headline `value`)."""
    res = {}
    gen = torch.Generator(device="cuda").manual_seed(7)
    # configs[3]: (4,16,8192,128) bf16 forward (+ backward when built)
    N, d, BH = 8192, 128, 64
    Q, K, V = (_randn_jl(fa_hip, (N, d, BH), torch.bfloat16, gen) for _ in range(3))
    O = fa_hip.jl_empty((N, d, BH), torch.bfloat16)
    l = fa_hip.jl_empty((N, 1, BH)); m = fa_hip.jl_empty((N, 1, BH))
    w, e = time_launches(lambda: fa_hip.dense_fa_(O, l, m, Q, K, V), max(3, args.steps // 2), 2, dist)
    f = 4.0 * BH * N * N * d
    res["cfg4_fwd_tflops"] = f / (e / max(3, args.steps // 2)) / 1e12
    try:
        dO = _randn_jl(fa_hip, (N, d, BH), torch.bfloat16, gen)
        steps = max(3, args.steps // 4)
        w, e = time_launches(lambda: fa_hip.dense_fa_backward(Q, K, V, O, dO, l, m), steps, 1, dist)
        res["cfg4_bwd_tflops"] = 2.5 * f / (e / steps) / 1e12
        res["cfg4_fwd_bwd_tflops"] = 3.5 * f / (e / steps + f / res["cfg4_fwd_tflops"] / 1e12) / 1e12
    except fa_hip.FlashAttentionError as ex:
        res["cfg4_bwd"] = str(ex)
    # configs[4]: (64,16,16384,128) over 8 GPUs -> this rank's share of 128 slabs
    N5, d5, BH5 = 16384, 128, 128
    Q5, K5, V5 = (_randn_jl(fa_hip, (N5, d5, BH5), torch.bfloat16, gen) for _ in range(3))
    O5 = fa_hip.jl_empty((N5, d5, BH5), torch.bfloat16)
    l5 = fa_hip.jl_empty((N5, 1, BH5)); m5 = fa_hip.jl_empty((N5, 1, BH5))
    w, e = time_launches(lambda: fa_hip.dense_fa_(O5, l5, m5, Q5, K5, V5), 3, 1, dist)
    res["cfg5_share_fwd_tflops_per_gpu"] = 4.0 * BH5 * N5 * N5 * d5 / (e / 3) / 1e12
    del Q5, K5, V5, O5
    # configs[2]: windowed 2-D bf16 128x128, ws=7, d=64 (B sweep)
    for Bimg in (1, 32):
        try:
            q, k, v = (_randn_jl(fa_hip, (128, 128, 64, Bimg), torch.bfloat16, gen) for _ in range(3))
            t = time_graph(lambda: fa_hip.windowed_fa(q, k, v, 7), args.steps, dist)
            T, L = 49, 19 * 19
            bytes_alg = Bimg * (3 * 128 * 128 * 64 * 2 + 128 * 128 * 64 * 2 + 2 * T * L * 4)
            res[f"cfg3_windowed_B{Bimg}_GBs"] = bytes_alg / t / 1e9
            res[f"cfg3_windowed_B{Bimg}_us"] = t * 1e6
            # backward of the same shape: q, k, v, y, dy read, dq, dk, dv written
            dy = _randn_jl(fa_hip, (128, 128, 64, Bimg), torch.bfloat16, gen)
            y, lw, mw = fa_hip.windowed_fa(q, k, v, 7)
            tb = time_graph(lambda: fa_hip.windowed_fa_backward(q, k, v, y, dy, lw, mw, 7), max(5, args.steps // 4), dist)
            bytes_bwd = Bimg * (8 * 128 * 128 * 64 * 2 + 2 * T * L * 4)
            res[f"cfg3_windowed_bwd_B{Bimg}_GBs"] = bytes_bwd / tb / 1e9
            res[f"cfg3_windowed_bwd_B{Bimg}_us"] = tb * 1e6
        except fa_hip.FlashAttentionError as ex:
            res[f"cfg3_windowed_B{Bimg}"] = str(ex)
    # circulant: the reference's runcirculant shape
    # (bench/compare.jl:105-115: N=4096, d=32, bs=1, W = 16..256) and a
    # device-scale shape (B·H=64, N=16384, d=64, W=129; HBM-bound, GB/s)
    for (Nc, dc, Bc, Wc) in ((4096, 32, 1, 16), (4096, 32, 1, 256), (16384, 64, 64, 129)):
        Qc, Kc, Vc = (_randn_jl(fa_hip, (Nc, dc, Bc), torch.bfloat16, gen) for _ in range(3))
        Oc = fa_hip.jl_empty((Nc, dc, Bc), torch.bfloat16)
        lc = fa_hip.jl_empty((Nc, 1, Bc)); mc = fa_hip.jl_empty((Nc, 1, Bc))
        t = time_graph(lambda: fa_hip.circulant_fa_(Oc, lc, mc, Qc, Kc, Vc, Wc), args.steps, dist)
        tag = f"circ_N{Nc}_d{dc}_B{Bc}_W{Wc}"
        res[f"{tag}_us"] = t * 1e6
        res[f"{tag}_GBs"] = Bc * Nc * (4 * dc * 2 + 8) / t / 1e9       # Q, K, V, O + l, m
        res[f"{tag}_tflops"] = 4.0 * Bc * Nc * Wc * dc / t / 1e12
    del Qc, Kc, Vc, Oc
    # fused softmax: a configs[1]-shaped score tensor
    # (4096 x 4096 x 64 bf16, 2 GiB) along each dim; HBM-bound: read + write
    Ssm = _randn_jl(fa_hip, (4096, 4096, 64), torch.bfloat16, gen)
    Psm = torch.empty_like(Ssm)
    for dims in (1, 2):
        steps = max(3, args.steps // 4)
        w, e = time_launches(lambda: fa_hip.fused_softmax_(Psm, Ssm, dims), steps, 1, dist)
        t = e / steps
        res[f"softmax_4096x4096x64_dims{dims}_GBs"] = 2 * Ssm.numel() * 2 / t / 1e9
        res[f"softmax_4096x4096x64_dims{dims}_us"] = t * 1e6
    return res


if __name__ == "__main__":
    main()
