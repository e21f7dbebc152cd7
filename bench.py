"""bench.py — headline benchmark (BASELINE.json metric).

metric : effective attention TFLOP/s (fwd) at N=4096, d=64; % of bf16 MFMA peak
step   : one fa_dense_fwd call over this rank's (B·H) slabs of BASELINE
         configs[1] = (B,H,N,d) = (4,16,4096,64) bf16, i.e. (N, d, B·H) =
         (4096, 64, 64) in the reference's column-major layout; inputs resident
         in HBM before the timed region.
FLOPs  : 4·(B·H)·N²·d per step per rank (non-causal; softmax not counted;
         SURVEY.md §8d).
scaling: weak — every rank processes its own 64 slabs (sharding over
         batch × head, no data-path collective; a barrier and a MAX
         all-reduce of the elapsed time are the only cross-rank calls).

Timing protocol:
  1. settle: the step is launched back-to-back, untimed, until >= --settle-ms of
     wall time has passed (default 250 ms).  From idle the GPU needs ~60 ms of
     load to reach its sustained clock; the settle phase is DISCLOSED in the JSON
     ("settle") together with the number measured without it ("cold": exactly W
     warm-up steps, then the same K timed steps, measured first).
  2. W untimed warm-up steps, then EXACTLY K timed steps bracketed by a barrier
     + torch.cuda.synchronize() on both sides; MAX over ranks.
  3. the GPU clock and board power are sampled (amdsmi via torch.cuda) during
     the timed region and reported ("clock").

Secondary blocks on the same JSON line (never the headline `value`), keyed by
the BASELINE.json configs index they measure:
  * "cfg2": configs[2] = windowed_fa 2-D bf16, 128x128 image, ws 7, d 64:
    forward and backward at B = 1 (as written) and B = 32, GB/s against the
    8 TB/s HBM roofline (HIP-graph replay: launch-bound at B = 1);
  * "cfg3": configs[3] = (4,16,8192,128) bf16 forward, backward and
    forward+backward TFLOP/s, each with its own MFMA roofline (2.5x / 3.5x the
    forward FLOPs), and whether the single-pass backward's dQ
    hand-off fell back (fa_dense_bwd_handoff_status);
  * "cfg4": configs[4] = (64,16,16384,128) bf16 forward, STRONG scaling: its
    1024 (B·H) slabs are split over the N ranks (fa_hip.shard.shard_range),
    each rank times its share; total TFLOP/s = all ranks' FLOPs / the slowest
    rank's time.
  * "cpu_baseline" (rank 0, N = 1): the reference's CPU algorithm
    (oracle/fa_cpu.c BLAS port of dense_fa!) on configs[0] at 1 thread and at
    the process's cores (median of 50 after 5 warm-ups), the reference's own
    published Float64 case (512, 64, 1) likewise, and the whole configs[1]
    workload (fp32).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu] [--no-cfg4] [--no-cfg23] [--extra]
Multi-GPU: `python bench.py --gpus N` (N > 1, WORLD_SIZE unset) starts N ranks
           itself as a child `python -m torch.distributed.run --nnodes=1
           --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N ...`
           (before any GPU call; the parent only waits and exits with the
           child's code, rank 0 prints the JSON line).  Launched by
           torch.distributed.run directly, --gpus must equal WORLD_SIZE
           (exit 2 otherwise).

Test hook (CPU only, never on a GPU run): FA_BENCH_CPU_STEP=1 replaces every
device step by a CPU stand-in (rank r sleeps (r + 1) * 5 ms per step) so that
tests/test_bench_dist.py can run the literal `python bench.py --gpus 2` with
FA_BENCH_BACKEND=gloo and check the launch, world, slab split and MAX
reduction; the JSON then says "cpu_step_hook": true.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import statistics
import sys
import threading
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
# BASELINE configs[4]: (B,H,N,d) = (64,16,16384,128), sharded over (B·H)
CFG4_SLABS, CFG4_N, CFG4_D = 64 * 16, 16384, 128


# ----------------------------------------------------------------------------
# process group / timing plumbing (device-agnostic: tests/test_bench_dist.py
# drives it with gloo on CPU)
# ----------------------------------------------------------------------------
def dist_init(backend: str | None = None):
    """One process per GPU; RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* from the
    env (torch.distributed.run).  backend: "nccl" (= RCCL) on GPUs, "gloo"
    for the CPU rehearsal.  Returns (dist or None, rank, world, local)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if backend is None:
        # FA_BENCH_BACKEND=gloo rehearses the multi-rank path on a one-GPU box
        # (every rank on cuda:0; RCCL refuses two ranks on one GPU)
        backend = os.environ.get("FA_BENCH_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    if backend == "nccl":
        torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
        return dist, rank, world, local
    return None, 0, 1, 0


def _cuda_sync():
    torch.cuda.synchronize()


def time_region(fn, steps, warmup, dist=None, sync=_cuda_sync, events=True):
    """W untimed calls, then exactly `steps` timed calls bracketed by a barrier
    + sync on both sides.  Returns (max-over-ranks wall s, max-over-ranks
    device-event s of the region; == wall without events)."""
    for _ in range(warmup):
        fn()
    sync()
    ev0 = ev1 = None
    if events:
        stream = torch.cuda.current_stream()
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
    if dist is not None:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    if events:
        ev0.record(stream)
    for _ in range(steps):
        fn()
    if events:
        ev1.record(stream)
    sync()
    if dist is not None:
        dist.barrier()
    wall = time.perf_counter() - t0
    ev_s = ev0.elapsed_time(ev1) / 1e3 if events else wall
    if dist is not None:
        t = torch.tensor([wall, ev_s], dtype=torch.float64,
                         device="cuda" if events else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall, ev_s = float(t[0]), float(t[1])
    return wall, ev_s


# kept for tools/ that import it
def time_launches(fn, steps, warmup, dist=None):
    return time_region(fn, steps, warmup, dist)


def settle(fn, min_s: float, sync=_cuda_sync):
    """Launch `fn` back-to-back (untimed) for at least min_s of wall time so the
    GPU leaves its idle clock before anything is timed.  Returns (launches, s)."""
    if min_s <= 0:
        return 0, 0.0
    t0 = time.perf_counter()
    n = 0
    while True:
        for _ in range(8):
            fn()
        n += 8
        sync()
        if time.perf_counter() - t0 >= min_s:
            return n, time.perf_counter() - t0


class ClockSampler:
    """Samples the GPU shader clock (MHz) and board power (W) through amdsmi
    (torch.cuda.clock_rate / power_draw) every ~1 ms on a host thread while a
    timed region runs.  Fields are None where the box does not expose them."""

    def __init__(self, device: int):
        self.device = device
        self.clk, self.pwr = [], []
        self._stop = threading.Event()
        self._th = None
        self.ok = True

    def _loop(self):
        while not self._stop.is_set():
            try:
                self.clk.append(float(torch.cuda.clock_rate(self.device)))
            except Exception:
                self.ok = False
                return
            try:
                self.pwr.append(float(torch.cuda.power_draw(self.device)))
            except Exception:
                pass
            time.sleep(0.001)

    def __enter__(self):
        self._th = threading.Thread(target=self._loop, daemon=True)
        self._th.start()
        return self

    def __exit__(self, *exc):
        self._stop.set()
        if self._th is not None:
            self._th.join(timeout=2.0)

    def summary(self):
        med = lambda xs: statistics.median(xs) if xs else None
        pw = med(self.pwr)
        if pw is not None and pw > 1e4:      # some amdsmi versions report microwatts
            pw = pw / 1e6
        return {"sclk_mhz_median": med(self.clk), "sclk_mhz_min": min(self.clk) if self.clk else None,
                "sclk_mhz_max": max(self.clk) if self.clk else None, "samples": len(self.clk),
                "power_w_median": pw, "source": "amdsmi (torch.cuda.clock_rate / power_draw)",
                "peak_at_measured_clock_tflops": (256 * med(self.clk) * 1e6 * 4096 / 1e12) if self.clk else None}


def sharded_strong(make_step, n_slabs_total: int, world: int, rank: int, dist, steps: int, warmup: int,
                   flops_per_slab: float, sync=_cuda_sync, events=True):
    """Strong scaling over (B·H) slabs: rank `rank` owns shard_range(n_slabs_total,
    world, rank) (contiguous slabs, sizes differ by <= 1), builds its step with
    make_step(n_local) and times it; no data-path collective.  Total throughput =
    every rank's FLOPs / the slowest rank's time (MAX all-reduce)."""
    from fa_hip.shard import shard_range
    a, b = shard_range(n_slabs_total, world, rank)
    n_local = b - a
    step = make_step(n_local)
    wall, ev_s = time_region(step, steps, warmup, dist, sync, events)
    per = ev_s / steps
    split = [shard_range(n_slabs_total, world, r) for r in range(world)]
    total_flops = flops_per_slab * n_slabs_total
    return {"slabs_total": n_slabs_total, "slab_split": [[x, y] for x, y in split],
            "slabs_this_rank": n_local, "steps": steps, "warmup": warmup,
            "ms_per_step_max_over_ranks": per * 1e3,
            "tflops_total": total_flops / per / 1e12,
            "tflops_per_gpu": total_flops / per / 1e12 / world,
            "frac_of_peak_per_gpu": total_flops / per / 1e12 / world / PEAK_BF16_TFLOPS,
            "scaling": "strong", "n_gpus": world}


# ----------------------------------------------------------------------------
# workloads
# ----------------------------------------------------------------------------
def _randn_jl(fa, shape, dtype, gen):
    t = fa.jl_empty(shape, dtype)
    t.normal_(generator=gen)
    return t


def cfg4_block(fa, world, rank, dist, steps, warmup, cpu_hook=False):
    """BASELINE configs[4]: dense_fa bf16 forward (N, d) = (16384, 128) over
    1024 (B·H) slabs, split over the ranks (strong scaling)."""
    N, d = CFG4_N, CFG4_D
    if cpu_hook:
        make_step = lambda n: _cpu_hook_step(rank)
        r = sharded_strong(make_step, CFG4_SLABS, world, rank, dist, steps, warmup, 4.0 * N * N * d,
                           sync=lambda: None, events=False)
    else:
        gen = torch.Generator(device="cuda").manual_seed(4242 + rank)

        def make_step(n):
            Q, K, V = (_randn_jl(fa, (N, d, n), torch.bfloat16, gen) for _ in range(3))
            O = fa.jl_empty((N, d, n), torch.bfloat16)
            l = fa.jl_empty((N, 1, n))
            m = fa.jl_empty((N, 1, n))
            return lambda: fa.dense_fa_(O, l, m, Q, K, V)

        r = sharded_strong(make_step, CFG4_SLABS, world, rank, dist, steps, warmup, 4.0 * N * N * d)
        torch.cuda.empty_cache()
    r["workload"] = "configs[4]: dense_fa bf16 forward, (B,H,N,d)=(64,16,16384,128), 1024 slabs split over ranks"
    r["kernel"] = "(cpu hook)" if cpu_hook else _fwd_kernel_128(fa)
    return r


def _fwd_kernel_128(fa):
    """The d = 128 forward kernel the last dense_fa_ call ran (fa_debug_fwd_last_path:
    30 = the one-wave-per-SIMD persistent kernel fa_fwd_p4.hip, else the 8-wave one)."""
    L = fa.lib()
    L.fa_debug_fwd_last_path.restype = ctypes.c_int
    return ("fa::dense_fwd_p4<bf16,128,128>" if L.fa_debug_fwd_last_path() == 30
            else "fa::dense_fwd_w8b64_wide<bf16,128,128>")


def _mfma_roofline(flops, seconds, kernel, note=None):
    ach = flops / seconds / 1e12
    r = {"bound": "mfma", "achieved": ach, "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
         "frac": ach / PEAK_BF16_TFLOPS, "kernel": kernel, "flops_per_launch": flops,
         "avg_launch_ms": seconds * 1e3}
    if note:
        r["note"] = note
    return r


def _traffic_json(kind: str, workload: str):
    """The newest committed PMC summary profiles/*<kind>_traffic*.json for `workload`
    (written from separate FETCH_SIZE / WRITE_SIZE rocprofv3 passes with the gfx950
    FETCH_SIZE x2 correction), or None."""
    import glob
    best = None
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", f"*{kind}_traffic*.json"))):
        try:
            j = json.load(open(p))
        except Exception:
            continue
        if j.get("workload", "").startswith(workload):
            best = j
    return best


def cfg3_block(fa, dist, steps_fwd=10, steps_bwd=5, settle_s=0.25):
    """BASELINE configs[3]: dense_fa bf16 (B,H,N,d) = (4,16,8192,128) forward,
    backward (reference src/dense.jl:104-167, executable spec
    src_cpp/FlashAttention.cpp:194-252) and forward+backward.  FLOPs: forward
    4·BH·N²·d, backward 2.5x, fwd+bwd 3.5x.  Device time by
    HIP events on the launch stream.  Each leg is timed twice: `*_cold` right
    after its warm-up calls, then again after `settle_s` of untimed back-to-back
    calls of the same leg (the configs[1] line's disclosed settle);
    the headline fields are the settled ones."""
    gen = torch.Generator(device="cuda").manual_seed(7)
    N, d, BH = 8192, 128, 64
    Q, K, V, dO = (_randn_jl(fa, (N, d, BH), torch.bfloat16, gen) for _ in range(4))
    O = fa.jl_empty((N, d, BH), torch.bfloat16)
    l = fa.jl_empty((N, 1, BH))
    m = fa.jl_empty((N, 1, BH))
    f = 4.0 * BH * N * N * d
    fwd = lambda: fa.dense_fa_(O, l, m, Q, K, V)
    _, e_fc = time_region(fwd, steps_fwd, 2, dist)
    n_sf, s_sf = settle(fwd, settle_s)
    _, e_f = time_region(fwd, steps_fwd, 0, dist)
    t_f, t_fc = e_f / steps_fwd, e_fc / steps_fwd
    k_f = _fwd_kernel_128(fa)
    fa.dense_fa_backward(Q, K, V, O, dO, l, m)   # the stream's scratch buffer exists before the count is read
    trips0 = fa.backward_handoff_trips(Q.device)
    bwd = lambda: fa.dense_fa_backward(Q, K, V, O, dO, l, m)
    _, e_bc = time_region(bwd, steps_bwd, 1, dist)
    n_sb, s_sb = settle(bwd, settle_s)
    _, e_b = time_region(bwd, steps_bwd, 0, dist)
    t_b, t_bc = e_b / steps_bwd, e_bc / steps_bwd
    hs = fa.backward_handoff_status(Q.device)   # the last timed call
    # slabs that gave up over the warm-up, settle and timed calls: a counter in the
    # workspace header that no call resets (fa_hip.backward_handoff_trips), read around them
    trips = (fa.backward_handoff_trips(Q.device) - trips0) & 0xFFFFFFFF
    rb = _mfma_roofline(
        2.5 * f, t_b, "fa::bwd_fused<bf16,128,128>",
        "whole fa_dense_bwd call (D = rowsum(dO*O) pre-pass + bwd_fused + the guarded dQ pass), "
        "FLOPs = 2.5x forward (the 5 GEMMs of the single pass)")
    tj = _traffic_json("bwd", "configs[3]")
    rb["traffic"] = tj.get("hbm_bytes_per_launch") if tj else None
    if tj:
        rb["traffic_over_algorithmic"] = tj.get("ratio_to_algorithmic")
        rb["traffic_source"] = "profiles/r06_bwd_traffic.json (rocprofv3 PMC, bwd_fused per launch)"
    res = {
        "workload": "configs[3]: dense_fa bf16 forward + backward, (B,H,N,d)=(4,16,8192,128)",
        "fwd_tflops": f / t_f / 1e12, "bwd_tflops": 2.5 * f / t_b / 1e12,
        "fwd_bwd_tflops": 3.5 * f / (t_f + t_b) / 1e12,
        "fwd_ms": t_f * 1e3, "bwd_ms": t_b * 1e3, "steps_fwd": steps_fwd, "steps_bwd": steps_bwd,
        "fwd_tflops_cold": f / t_fc / 1e12, "bwd_tflops_cold": 2.5 * f / t_bc / 1e12,
        "fwd_ms_cold": t_fc * 1e3, "bwd_ms_cold": t_bc * 1e3,
        "settle": {"fwd_launches": n_sf, "fwd_ms": s_sf * 1e3, "bwd_launches": n_sb, "bwd_ms": s_sb * 1e3},
        "roofline_fwd": _mfma_roofline(f, t_f, k_f),
        "roofline_bwd": rb,
        "roofline_fwd_bwd": _mfma_roofline(3.5 * f, t_f + t_b, "forward + backward calls"),
        "bwd_handoff": {-1: "two-pass plan (no hand-off)", 0: "single pass, hand-off completed",
                        1: "single pass, a slab's hand-off GAVE UP (the launch made no progress for 100 ms): its dQ recomputed by the guarded pass"}.get(hs, hs),
        "bwd_handoff_giveups": trips,
        "bwd_fallback_tainted": trips != 0 or hs == 1,
    }
    del Q, K, V, dO, O, l, m
    torch.cuda.empty_cache()
    return res


def cfg2_block(fa, dist, steps=20):
    """BASELINE configs[2]: windowed_fa 2-D bf16, 128x128 image, ws 7 (stride 7,
    pad 3: 19x19 windows of 49 tokens), d 64 (reference src/windowed.jl:3-23,
    src/utils.jl:36-54); forward and backward at B = 1 (as written) and
    B = 32.  HBM-bound (26 FLOP/B): algorithmic bytes = q, k, v read + y
    written (+ l, m) for the forward; q, k, v, dy read + dq, dk, dv written
    (+ l, m) for the backward (y is not needed: the strip backward forms
    D = rowsum(P ∘ dP); the one-window kernel still reads it); GB/s against 8 TB/s.
    Kernels: B = 1 runs the per-window kernels, B = 32 the strip kernels
    (>= 256 strips)."""
    gen = torch.Generator(device="cuda").manual_seed(11)
    T, L, S, dd = 49, 19 * 19, 128 * 128, 64
    res = {"workload": "configs[2]: windowed_fa 2-D bf16, 128x128 image, ws=7, d=64, stride 7, pad 3",
           "timing": "HIP-graph replay of back-to-back calls (device time per call)"}
    for Bimg in (1, 32):
        q, k, v, dy = (_randn_jl(fa, (128, 128, dd, Bimg), torch.bfloat16, gen) for _ in range(4))
        t = time_graph(lambda: fa.windowed_fa(q, k, v, 7), steps, dist)
        by = Bimg * (4 * S * dd * 2 + 2 * T * L * 4)
        y, lw, mw = fa.windowed_fa(q, k, v, 7)
        tb = time_graph(lambda: fa.windowed_fa_backward(q, k, v, y, dy, lw, mw, 7), max(5, steps // 2), dist)
        bb = Bimg * (7 * S * dd * 2 + 2 * T * L * 4)
        res[f"B{Bimg}"] = {
            "fwd_us": t * 1e6, "fwd_GBs": by / t / 1e9, "fwd_frac_hbm": by / t / 1e9 / PEAK_HBM_GBS,
            "fwd_bytes": by,
            "fwd_kernel": "fa::win_strip<bf16,64,64>" if Bimg >= 5 else "fa::win_rows1s<bf16,64,64,2>",
            "bwd_us": tb * 1e6, "bwd_GBs": bb / tb / 1e9, "bwd_frac_hbm": bb / tb / 1e9 / PEAK_HBM_GBS,
            "bwd_bytes": bb,
            "bwd_kernel": "fa::win_bwd_strip<bf16,64,64>" if Bimg >= 5 else "fa::win_bwd_rows<bf16,64,64,2>"}
        del q, k, v, dy, y, lw, mw
    torch.cuda.empty_cache()
    return res


def _cpu_hook_step(rank):
    """FA_BENCH_CPU_STEP=1 stand-in for a device step (tests only): rank r
    sleeps (r + 1) * 5 ms, so the MAX over ranks is the last rank's time."""
    return lambda: time.sleep(0.005 * (rank + 1))


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def _cpu_threads():
    """Cores this process may use: its affinity set, capped by the box's
    OMP_NUM_THREADS share when set (the GPU box exports 16 per GPU)."""
    n = _node_cpus()
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        n = min(n, int(env))
    return max(1, n)


def _cpu_quota():
    """The cgroup CPU quota of this process (cpu.max: quota / period), or None."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        return None


def _node_cpus():
    """Every host CPU this process may run on (sched_getaffinity): the node's
    cores as north_star's CPU baseline asks for."""
    return len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)


def _plain_port(Q, K, V, nthreads):
    """oracle/fa_cpu.c's OpenMP port of dense_fa! without BLAS (same tiles, scalar
    / SIMD loops), for thread counts past numpy's OpenBLAS build limit."""
    import ctypes
    import numpy as np
    from oracle import cpu_port
    N, d, B = Q.shape
    O = np.empty((N, V.shape[1], B), np.float32, order="F")
    l = np.empty((N, 1, B), np.float32, order="F")
    m = np.empty((N, 1, B), np.float32, order="F")
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    rc = cpu_port.lib().fa_cpu_dense_fwd_f32(p(Q), p(K), p(V), p(O), p(l), p(m), N, K.shape[0], d, V.shape[1], B,
                                             int(nthreads))
    if rc != 0:
        raise RuntimeError(f"fa_cpu_dense_fwd_f32 failed ({rc})")
    return O


# numpy's OpenBLAS is built with MAX_THREADS=64: more concurrent single-threaded sgemm
# callers than its buffer table holds corrupt its allocator ("Bad memory unallocation")
OPENBLAS_MAX_CALLERS = 64


def cpu_baseline(node: bool = False):
    """The reference's CPU algorithm, dense_fa! (src/dense.jl:21-102), as the
    BLAS-backed C/OpenMP port oracle/fa_cpu.c (same Br/Bc tiles, one gemm per
    tile product, (slab x row-block) tasks), fp32.
      * default leg "share": the box's per-GPU OMP_NUM_THREADS share (16 on the GPU
        box; the harness asks GPU jobs to keep their worker pools to it) -> `value`;
      * node=True (bench.py --cpu-node) adds the node's host cores, every CPU of the
        affinity set (north_star): "node_blas" = the BLAS port at min(CPUs, 64)
        threads (numpy's OpenBLAS build limit), "node_plain" = the same algorithm
        without BLAS on all CPUs; `value` / `cores` then come from the faster leg.
    Each leg times configs[0] (N,d,B·H) = (512,64,4) (median of 50 after 5
    warm-ups; also at 1 thread), the reference's own published Float64 case
    (512,64,1) (logs/compare1.txt:4), and the whole configs[1] workload
    (4096,64,64) (median of 3 after 1 warm-up)."""
    import numpy as np
    from oracle import cpu_port
    cpu_port.blas_info()
    ncpu, share = _node_cpus(), _cpu_threads()
    rng = np.random.default_rng(0)

    def arrs(N, d, n, dt=np.float32):
        return [np.asfortranarray(rng.standard_normal((N, d, n)).astype(dt)) for _ in range(3)]

    def med_time(fn, reps, warm):
        for _ in range(warm):
            fn()
        ts = []
        for _ in range(reps):
            t = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t)
        return statistics.median(ts)

    q0, k0, v0 = arrs(512, 64, 4)
    qr, kr, vr = arrs(512, 64, 1, np.float64)
    q1, k1, v1 = arrs(N_, D_, B_ * H_)
    f0, fr, f1 = 4.0 * 4 * 512 * 512 * 64, 4.0 * 512 * 512 * 64, 4.0 * B_ * H_ * N_ * N_ * D_
    legs = {}
    plan = [("share", share, "blas")]
    if node:
        plan += [("node_blas", min(ncpu, OPENBLAS_MAX_CALLERS), "blas"), ("node_plain", ncpu, "plain")]
    for tag, th, kind in plan:
        run = (lambda q, k, v, t_: cpu_port.dense_fa_blas(q, k, v, t_)) if kind == "blas" else _plain_port
        c0 = {}
        for t_ in sorted({1, th}):
            t = med_time(lambda: run(q0, k0, v0, t_), 50, 5)
            c0[f"threads_{t_}"] = {"ms": t * 1e3, "gflops": f0 / t / 1e9}
        leg = {"threads": th, "impl": "BLAS port (OpenBLAS sgemm per tile product)" if kind == "blas"
               else "OpenMP port without BLAS", "configs0_fp32_512x64x4": c0}
        if kind == "blas":
            tr = med_time(lambda: cpu_port.dense_fa_blas(qr, kr, vr, th), 50, 5)
            leg["reference_case_f64_512x64x1"] = {"ms": tr * 1e3, "gflops": fr / tr / 1e9}
        t1 = med_time(lambda: run(q1, k1, v1, th), 3, 1)
        leg.update(configs1_fp32_tflops=f1 / t1 / 1e12, configs1_s=t1)
        legs[tag] = leg
    best = max(legs, key=lambda t: legs[t]["configs1_fp32_tflops"])
    bl = legs[best]
    return {"value": bl["configs1_fp32_tflops"], "unit": "TFLOP/s", "cores": bl["threads"], "kind": "port",
            "value_from": best, "cpu_model": _cpu_model(), "affinity_cpus": ncpu, "omp_share": share,
            "cgroup_cpu_quota": _cpu_quota(),
            "sample": f"the whole configs[1] workload (4096,64,64) fp32, C/OpenMP port of dense_fa! "
                      f"(oracle/fa_cpu.c: Br=64 Bc=500 tiles), leg '{best}': {bl['impl']} at {bl['threads']} "
                      f"threads, median of 3: {bl['configs1_s']:.3f} s; 'legs' adds configs[0] and the "
                      f"reference's Float64 case" + ("" if node else
                      f"; the node-wide legs (all {ncpu} affinity CPUs) run with bench.py --cpu-node "
                      f"(profiles/r04_cpu_baseline_node.log: slower than this leg, since the job's "
                      f"cgroup quota is {_cpu_quota()} CPUs)"),
            "legs": legs,
            "reference_published": "dense_fa Julia N=512 d=64 bs=1 Float64: 2.392 ms, unstated CPU "
                                   "(/root/reference/logs/compare1.txt:4)"}


def _traffic_from_profiles():
    """HBM bytes per launch of the configs[1] forward kernel from the committed
    rocprofv3 PMC summary (profiles/*fwd_traffic*.json, written by
    profiles/pmc_traffic.py)."""
    j = _traffic_json("fwd", "configs[1]")
    return j.get("hbm_bytes_per_launch") if j else None


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int, argv) -> int:
    """`bench.py --gpus N` without a torch.distributed.run environment: start
    the N ranks as ONE child process tree (python -m torch.distributed.run,
    rendezvous on 127.0.0.1) and return its exit code.  Called before anything
    touches the GPU; the parent never re-execs itself, it only waits (rank 0's
    JSON line reaches stdout directly)."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--settle-ms", type=float, default=250.0,
                    help="untimed back-to-back launches before timing (disclosed in the JSON)")
    ap.add_argument("--cfg4-steps", type=int, default=3)
    ap.add_argument("--no-cpu", action="store_true", help="skip the cpu_baseline leg")
    ap.add_argument("--cpu-node", action="store_true",
                    help="cpu_baseline also on every affinity CPU (beyond the box's per-GPU share)")
    ap.add_argument("--no-cfg4", action="store_true", help="skip the configs[4] strong-scaling block")
    ap.add_argument("--no-cfg23", action="store_true", help="skip the configs[2] / configs[3] blocks")
    ap.add_argument("--no-cfg2", action="store_true", help="skip the configs[2] block")
    ap.add_argument("--no-cfg3", action="store_true", help="skip the configs[3] block")
    ap.add_argument("--extra", action="store_true", help="also time the secondary paths (reported under 'extra')")
    args = ap.parse_args()
    if args.gpus < 1:
        print(f"bench.py: --gpus must be >= 1 (got {args.gpus})", file=sys.stderr)
        return 2
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch_ranks(args.gpus, sys.argv[1:])
    env_world = int(os.environ.get("WORLD_SIZE", "1"))
    if env_world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={env_world}: launch one rank per GPU "
              f"(torch.distributed.run --nproc-per-node {args.gpus}) or drop --gpus", file=sys.stderr)
        return 2

    cpu_hook = os.environ.get("FA_BENCH_CPU_STEP") == "1"
    if cpu_hook and torch.cuda.is_available():
        print("bench.py: FA_BENCH_CPU_STEP is a CPU test hook; refusing it on a GPU box", file=sys.stderr)
        return 2
    dist, rank, world, local = dist_init("gloo" if cpu_hook else None)
    # the one-GPU rehearsal (FA_BENCH_BACKEND=gloo): every rank on cuda:0
    shared_gpu = (not cpu_hook and world > 1 and os.environ.get("FA_BENCH_BACKEND") == "gloo"
                  and torch.cuda.is_available())

    if cpu_hook:
        fa_hip = None
        step = _cpu_hook_step(rank)
        sync, events = (lambda: None), False
    else:
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
        sync, events = _cuda_sync, True
    BH = B_ * H_
    flops_rank = 4.0 * BH * N_ * N_ * D_
    sampler = (lambda: _NullSampler()) if cpu_hook else (lambda: ClockSampler(torch.cuda.current_device()))

    # cold: exactly W warm-up steps from idle, then the K timed steps
    wall_c, ev_c = time_region(step, args.steps, args.warmup, dist, sync, events)
    with sampler() as clk_settle:   # sustained load: many samples
        settle_n, settle_s = settle(step, (0.0 if cpu_hook else args.settle_ms) / 1e3, sync)
    with sampler() as clk:
        wall, ev_s = time_region(step, args.steps, args.warmup, dist, sync, events)
    value = flops_rank * world * args.steps / wall / 1e12
    kern_s = ev_s / args.steps
    achieved = flops_rank / kern_s / 1e12

    out = {
        "metric": METRIC, "value": value, "unit": "TFLOP/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": wall / args.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
        "data": "synthetic (torch normal_ -> bf16, column-major (N,d,B*H) device arrays)",
        "config": {"workload": "configs[1]: dense_fa bf16 forward, (B,H,N,d)=(4,16,4096,64) per GPU",
                   "B": B_, "H": H_, "N": N_, "d": D_, "slabs_per_gpu": BH,
                   "global_batch_heads": BH * world, "parallelism": f"shard(B*H) x{world}, no collective"},
        "roofline": {"bound": "mfma", "achieved": achieved, "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                     "frac": achieved / PEAK_BF16_TFLOPS, "traffic": _traffic_from_profiles(),
                     "kernel": "fa::dense_fwd_w8q2_wide<bf16,64,64>",
                     "flops_per_launch": flops_rank, "avg_launch_ms": kern_s * 1e3},
        "settle": {"ms": settle_s * 1e3, "launches": settle_n,
                   "why": "untimed back-to-back launches so the GPU leaves its idle clock (DESIGN.md §6)"},
        "cold": {"value": flops_rank * world * args.steps / wall_c / 1e12,
                 "avg_launch_ms": ev_c / args.steps * 1e3,
                 "what": "the same K steps after exactly W warm-up steps from idle, measured before settle"},
        "clock": clk.summary(),
        # the timed region lasts a few ms, which holds one or two amdsmi samples (and the
        # power reading averages over a longer window): the settle phase just before it
        # runs the same launches back to back for --settle-ms and is sampled throughout
        "clock_settle": clk_settle.summary(),
    }
    if cpu_hook:
        out["cpu_step_hook"] = True

    # configs[2] (HBM-bound, microseconds per call) before the d = 128 blocks, whose
    # sustained 1400-W load would otherwise set the clock it is timed at
    if not (args.no_cfg23 or args.no_cfg2) and not cpu_hook:
        out["cfg2"] = cfg2_block(fa_hip, dist)
    if not (args.no_cfg23 or args.no_cfg3) and not cpu_hook:
        out["cfg3"] = cfg3_block(fa_hip, dist, settle_s=args.settle_ms / 1e3)
        if shared_gpu:
            # co-tenant ranks: the single pass needs no co-residency (every hand-off wait
            # is on an earlier-dispatched workgroup), so it stays the plan here too
            out["cfg3"]["bwd_plan"] = "single pass: the ranks share one GPU"
    if not args.no_cfg4:
        out["cfg4"] = cfg4_block(fa_hip, world, rank, dist, args.cfg4_steps, 1, cpu_hook)

    if args.extra and not cpu_hook:
        out["extra"] = extra_benches(fa_hip, args, dist)

    if rank == 0 and world == 1 and not args.no_cpu and not cpu_hook:
        out["cpu_baseline"] = cpu_baseline(node=args.cpu_node)
    elif rank == 0:
        out["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    return 0


class _NullSampler:
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False

    def summary(self):
        return None


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
    _, e = time_region(graph.replay, 3, 1, dist)
    return e / 3 / steps


def extra_benches(fa_hip, args, dist):
    """Secondary BASELINE configs (not the headline `value`)."""
    res = {}
    gen = torch.Generator(device="cuda").manual_seed(7)
    # configs[3]: (4,16,8192,128) bf16 forward + backward
    N, d, BH = 8192, 128, 64
    Q, K, V = (_randn_jl(fa_hip, (N, d, BH), torch.bfloat16, gen) for _ in range(3))
    O = fa_hip.jl_empty((N, d, BH), torch.bfloat16)
    l = fa_hip.jl_empty((N, 1, BH)); m = fa_hip.jl_empty((N, 1, BH))
    st = max(3, args.steps // 2)
    w, e = time_region(lambda: fa_hip.dense_fa_(O, l, m, Q, K, V), st, 2, dist)
    f = 4.0 * BH * N * N * d
    res["cfg4_fwd_tflops"] = f / (e / st) / 1e12
    dO = _randn_jl(fa_hip, (N, d, BH), torch.bfloat16, gen)
    steps = max(3, args.steps // 4)
    w, e = time_region(lambda: fa_hip.dense_fa_backward(Q, K, V, O, dO, l, m), steps, 1, dist)
    res["cfg4_bwd_tflops"] = 2.5 * f / (e / steps) / 1e12
    res["cfg4_fwd_bwd_tflops"] = 3.5 * f / (e / steps + f / res["cfg4_fwd_tflops"] / 1e12) / 1e12
    del Q, K, V, O, dO
    # configs[2]: windowed 2-D bf16 128x128, ws=7, d=64 (B sweep)
    for Bimg in (1, 32):
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
    # Float64 dense forward on the reference's own published cases
    # (logs/compare1.txt:4,7: Julia Float64 CPU dense_fa at N=512 / 4096, d=64,
    # bs=1: 2.392 / 28.64 ms) and on configs[0] (B·H = 4)
    for (Nf, Bf) in ((512, 1), (512, 4), (4096, 1)):
        Qf, Kf, Vf = (_randn_jl(fa_hip, (Nf, 64, Bf), torch.float64, gen) for _ in range(3))
        Of = fa_hip.jl_empty((Nf, 64, Bf), torch.float64)
        lf = fa_hip.jl_empty((Nf, 1, Bf)); mf = fa_hip.jl_empty((Nf, 1, Bf))
        t = time_graph(lambda: fa_hip.dense_fa_(Of, lf, mf, Qf, Kf, Vf), args.steps, dist)
        res[f"f64_dense_N{Nf}_d64_B{Bf}_us"] = t * 1e6
        res[f"f64_dense_N{Nf}_d64_B{Bf}_gflops"] = 4.0 * Bf * Nf * Nf * 64 / t / 1e9
    # the reference's runwindow benchmark (bench/compare.jl:105-115: 1-D windowed_fa,
    # N = 4096, d = 32, bs = 1, stride 8, pad 0, Float64; logs/wind_t16.txt at 16
    # threads: W = 16 / 128 / 512 -> 10.4 / 115.1 / 805.0 ms), in Float64 and bf16
    for Ww in (16, 128, 512):
        for dt, tag in ((torch.float64, "f64"), (torch.bfloat16, "bf16")):
            qw, kw, vw = (_randn_jl(fa_hip, (4096, 32, 1), dt, gen) for _ in range(3))
            t = time_graph(lambda: fa_hip.windowed_fa(qw, kw, vw, Ww, stride=8, pad=0), max(5, args.steps // 4), dist)
            res[f"runwindow_W{Ww}_{tag}_us"] = t * 1e6
    # fused softmax: a configs[1]-shaped score tensor
    # (4096 x 4096 x 64 bf16, 2 GiB) along each dim; HBM-bound: read + write
    Ssm = _randn_jl(fa_hip, (4096, 4096, 64), torch.bfloat16, gen)
    Psm = torch.empty_like(Ssm)
    for dims in (1, 2):
        steps = max(3, args.steps // 4)
        w, e = time_region(lambda: fa_hip.fused_softmax_(Psm, Ssm, dims), steps, 1, dist)
        t = e / steps
        res[f"softmax_4096x4096x64_dims{dims}_GBs"] = 2 * Ssm.numel() * 2 / t / 1e9
        res[f"softmax_4096x4096x64_dims{dims}_us"] = t * 1e6
    return res


if __name__ == "__main__":
    sys.exit(main())
