"""A/B two (or more) builds of libfa_hip.so in ONE process, interleaved rounds:
dense forward at configs[1] and configs[3]-fwd, and circulant at
(64, 16384, 64, W=129).  Usage: python tools/ab_lib.py LIB_A LIB_B ..."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import numpy as np, torch
import fa_hip

paths = sys.argv[1:]
libs = []
for p in paths:
    fa_hip._LIB = None
    os.environ["FA_HIP_LIB"] = os.path.abspath(p)
    libs.append(fa_hip.lib())
PEAK = 2516.58


def mk(shape, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    out = []
    for _ in range(3):
        t = fa_hip.jl_empty(shape, torch.bfloat16)
        t.copy_(torch.randn(shape, generator=g, device="cuda"))
        out.append(t)
    return out


def bench(name, fn, flops):
    outs = []
    for L in libs:
        fa_hip._LIB = L
        outs.append([x.clone() for x in fn()])
        torch.cuda.synchronize()
    for i in range(1, len(libs)):
        same = all(torch.equal(a, b) for a, b in zip(outs[0], outs[i]))
        diff = max((a.float() - b.float()).abs().max().item() for a, b in zip(outs[0], outs[i]))
        print(f"{name}: lib{i} vs lib0 bitwise equal={same} max|diff|={diff:.3e}", flush=True)
    times = [[] for _ in libs]
    fa_hip._LIB = libs[0]
    for _ in range(400):   # past the clock ramp (tools/exp/ramp.py: ~200 launches)
        fn()
    for rnd in range(int(os.environ.get("AB_ROUNDS", 8))):
        for i, L in enumerate(libs):
            fa_hip._LIB = L
            for _ in range(2):
                fn()
            e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                fn()
            e1.record(); torch.cuda.synchronize()
            times[i].append(e0.elapsed_time(e1) / 10 / 1e3)
    for i, p in enumerate(paths):
        t = np.median(times[i])
        print(f"{name} {os.path.basename(p)}: {t*1e6:.1f} us  {flops/t/1e12:.1f} TFLOP/s "
              f"({flops/t/1e12/PEAK*100:.1f}%)  min {min(times[i])*1e6:.1f} us", flush=True)


for (N, d, BH) in [(4096, 64, 64), (8192, 128, 64)]:
    Q, K, V = mk((N, d, BH), 1)
    O_ = fa_hip.jl_empty((N, d, BH), torch.bfloat16)
    l = fa_hip.jl_empty((N, 1, BH)); m = fa_hip.jl_empty((N, 1, BH))

    def fwd():
        fa_hip.dense_fa_(O_, l, m, Q, K, V)
        return O_, l, m
    bench(f"dense N={N} d={d}", fwd, 4.0 * BH * N * N * d)
    del Q, K, V, O_

if os.environ.get("AB_BWD"):   # dense backward (configs[3] and d = 64) and windowed forward / backward at B = 32
    for (N, d, BH) in [(8192, 128, 64), (4096, 64, 64)]:
        Q, K, V = mk((N, d, BH), 3)
        dO = mk((N, d, BH), 4)[0]
        O_, l, m = fa_hip.dense_fa(Q, K, V)

        def bwd():
            return fa_hip.dense_fa_backward(Q, K, V, O_, dO, l, m)
        bench(f"dense bwd N={N} d={d}", bwd, 2.5 * 4.0 * BH * N * N * d)
        del Q, K, V, dO, O_
    q, k, v, dy = (fa_hip.jl_tensor(torch.randn((128, 128, 64, 32), device="cuda"), torch.bfloat16) for _ in range(4))
    bench("windowed fwd B=32", lambda: fa_hip.windowed_fa(q, k, v, 7), 1.0)
    y, lw, mw = fa_hip.windowed_fa(q, k, v, 7)
    bench("windowed bwd B=32", lambda: fa_hip.windowed_fa_backward(q, k, v, y, dy, lw, mw, 7), 1.0)

if os.environ.get("AB_DENSE_ONLY"):
    sys.exit(0)
N, d, BH, W = 16384, 64, 64, 129
Q, K, V = mk((N, d, BH), 2)
O_ = fa_hip.jl_empty((N, d, BH), torch.bfloat16)
l = fa_hip.jl_empty((N, 1, BH)); m = fa_hip.jl_empty((N, 1, BH))


def circ():
    fa_hip.circulant_fa_(O_, l, m, Q, K, V, W)
    return O_, l, m
bench("circulant W=129", circ, 4.0 * BH * N * W * d)
