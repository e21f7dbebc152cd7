"""Run a workload back-to-back for a few seconds while sampling the GPU's clock
and power with rocm-smi in child processes: tells whether a kernel is
power/clock-capped (DVFS) or issue-bound at full clock.  Prints TFLOP/s, the mean
of the power and sclk samples, and the energy per FLOP (pJ/FLOP = W / FLOP/s) so
kernels can be compared at the board's power cap.
Usage: python tools/power_probe.py [seconds] [fwd|fwd128|gemm|bwd]..."""
import os, subprocess, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import torch
import fa_hip

secs = float(sys.argv[1]) if len(sys.argv) > 1 else 6.0
modes = sys.argv[2:] or ["fwd"]
g = torch.Generator(device="cuda").manual_seed(0)


def jl(shape):
    t = fa_hip.jl_empty(shape, torch.bfloat16)
    t.copy_(torch.randn(shape, generator=g, device="cuda"))
    return t


def workload(mode):
    if mode in ("fwd", "fwd128", "bwd"):
        N, d, BH = (4096, 64, 64) if mode == "fwd" else (8192, 128, 64)
        Q, K, V = jl((N, d, BH)), jl((N, d, BH)), jl((N, d, BH))
        O = fa_hip.jl_empty((N, d, BH), torch.bfloat16)
        l = fa_hip.jl_empty((N, 1, BH)); m = fa_hip.jl_empty((N, 1, BH))
        fa_hip.dense_fa_(O, l, m, Q, K, V)
        if mode == "bwd":
            dO = jl((N, d, BH))
            return (lambda: fa_hip.dense_fa_backward(Q, K, V, O, dO, l, m)), 10.0 * BH * N * N * d
        return (lambda: fa_hip.dense_fa_(O, l, m, Q, K, V)), 4.0 * BH * N * N * d
    n = 8192
    a = torch.randn((n, n), device="cuda", dtype=torch.bfloat16)
    b = torch.randn((n, n), device="cuda", dtype=torch.bfloat16)
    c = torch.empty((n, n), device="cuda", dtype=torch.bfloat16)
    return (lambda: torch.matmul(a, b, out=c)), 2.0 * n ** 3


def smi():
    return subprocess.Popen(["rocm-smi", "--showpower", "--showclocks"],
                            stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)


def parse(txt):
    """(watts, MHz) of one rocm-smi sample (None where absent)."""
    pw = [l.split(":")[-1].strip() for l in txt.splitlines() if "Power (W)" in l]
    sc = [l.split("(")[-1].rstrip(")").lower().replace("mhz", "") for l in txt.splitlines() if "sclk" in l]
    f = lambda v: float(v[0]) if v else None
    try:
        return f(pw), f(sc)
    except ValueError:
        return None, None


for mode in modes:
    fn, flops = workload(mode)
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    t_end = time.time() + secs
    n, probes, next_probe = 0, [], time.time() + secs / 4
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    while time.time() < t_end:
        for _ in range(10):
            fn()
        n += 10
        if time.time() > next_probe and len(probes) < 3:
            probes.append(smi())
            next_probe += secs / 5
    e1.record(); torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / 1e3 / n
    samples = [parse(p.communicate(timeout=60)[0]) for p in probes]
    w = [a for a, _ in samples if a is not None]
    mhz = [b for _, b in samples if b is not None]
    tf = flops / t / 1e12
    wm = sum(w) / len(w) if w else float("nan")
    mm = sum(mhz) / len(mhz) if mhz else float("nan")
    print(f"{mode}: {n} launches, {t*1e6:.1f} us each, {tf:.1f} TFLOP/s | power {wm:.0f} W, sclk {mm:.0f} MHz, "
          f"{wm / (tf * 1e12) * 1e12:.3f} pJ/FLOP | samples {samples}", flush=True)
    del fn
    torch.cuda.empty_cache()
    time.sleep(2)
