"""A/B the dense backward of two (or more) builds of libfa_hip.so in ONE process,
interleaved rounds after a clock settle; each build is checked against the oracle on
one slab and bitwise against the first build.
Usage: python tools/ab_bwd_libs.py LIB_A LIB_B ... [--shapes N,d,BH ...]"""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import numpy as np, torch
import fa_hip
from oracle import fa_oracle as O

PEAK = 2516.58
args = sys.argv[1:]
paths, shapes = [], [(8192, 128, 64), (4096, 64, 64)]
while args:
    a = args.pop(0)
    if a == "--shapes":
        shapes = []
        while args and "," in args[0]:
            shapes.append(tuple(int(x) for x in args.pop(0).split(",")))
    else:
        paths.append(a)
libs = []
for p in paths:
    fa_hip._LIB = None
    os.environ["FA_HIP_LIB"] = os.path.abspath(p)
    libs.append(fa_hip.lib())
    # AB_MODE=m: fa_debug_set_bwd_mode(m) in every build (4.. = timing-only ablations of -DFA_BWD_ABL builds)
    if os.environ.get("AB_MODE") is not None:
        libs[-1].fa_debug_set_bwd_mode(int(os.environ["AB_MODE"]))
    # AB_L2LOCAL=0/1: force the single pass's L2-local hand-off form in every build
    if os.environ.get("AB_L2LOCAL") is not None and hasattr(libs[-1], "fa_debug_set_bwd_l2local"):
        libs[-1].fa_debug_set_bwd_l2local(int(os.environ["AB_L2LOCAL"]))
    # AB_HOFF=k: the single pass's chain step offset in every build
    if os.environ.get("AB_HOFF") is not None:
        libs[-1].fa_debug_set_bwd_hoff(int(os.environ["AB_HOFF"]))
rounds = int(os.environ.get("AB_ROUNDS", 6))
for (N, d, BH) in shapes:
    g = torch.Generator(device="cuda").manual_seed(1)
    mk = lambda: fa_hip.jl_tensor(torch.randn((N, d, BH), generator=g, device="cuda"), torch.bfloat16)
    Q, K, V, dO = mk(), mk(), mk(), mk()
    fa_hip._LIB = libs[0]
    Oo, l, m = fa_hip.dense_fa(Q, K, V)
    torch.cuda.synchronize()
    sl = lambda t: t[:, :, :1].float().cpu().double().numpy()
    ref = O.dense_fa_backward(sl(Q), sl(K), sl(V), sl(Oo), sl(dO), l[:, :, :1].cpu().double().numpy(),
                              m[:, :, :1].cpu().double().numpy())
    fl = 4.0 * BH * N * N * d * 2.5
    outs = []
    for i, L in enumerate(libs):
        fa_hip._LIB = L
        outs.append([x.clone() for x in fa_hip.dense_fa_backward(Q, K, V, Oo, dO, l, m)])
        again = fa_hip.dense_fa_backward(Q, K, V, Oo, dO, l, m)
        torch.cuda.synchronize()
        errs = [float(np.abs(sl(x) - y).max() / np.abs(y).max()) for x, y in zip(outs[i], ref)]
        same = all(torch.equal(a, b) for a, b in zip(outs[i], outs[0]))
        rep = all(torch.equal(a, b) for a, b in zip(outs[i], again))
        print(f"N={N} d={d} BH={BH} lib{i}: rel err dQ/dK/dV {errs[0]:.2e} {errs[1]:.2e} {errs[2]:.2e}  "
              f"bitwise vs lib0: {same}  repeatable: {rep}", flush=True)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:
        fa_hip.dense_fa_backward(Q, K, V, Oo, dO, l, m)
        torch.cuda.synchronize()
    ts = [[] for _ in libs]
    for rnd in range(rounds):
        for i, L in enumerate(libs):
            fa_hip._LIB = L
            fa_hip.dense_fa_backward(Q, K, V, Oo, dO, l, m)
            e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3):
                fa_hip.dense_fa_backward(Q, K, V, Oo, dO, l, m)
            e1.record(); torch.cuda.synchronize()
            ts[i].append(e0.elapsed_time(e1) / 3 / 1e3)
    for i, p in enumerate(paths):
        t = float(np.median(ts[i]))
        print(f"N={N} d={d} BH={BH} {os.path.basename(p)}: {t*1e3:.3f} ms  {fl/t/1e12:.1f} TFLOP/s "
              f"(2.5x convention, {fl/t/1e12/PEAK*100:.1f}% peak)  best {fl/min(ts[i])/1e12:.1f}", flush=True)
