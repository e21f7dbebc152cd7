"""A/B the backward MFMA paths in ONE process (interleaved rounds after a clock
settle): mode 1 = dK/dV pass + dQ pass (7 products), mode 2 = single pass
(5 products, ordered dQ hand-off).  Checks each against the oracle on one slab.
Usage: python tools/ab_bwd.py [--shapes N,d,BH ...] [modes...]"""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import numpy as np, torch
import fa_hip
from oracle import fa_oracle as O
L = fa_hip.lib()
PEAK = 2516.58
args = sys.argv[1:]
shapes = [(8192, 128, 64), (4096, 64, 64)]
if args and args[0] == "--shapes":
    shapes = []
    args = args[1:]
    while args and "," in args[0]:
        shapes.append(tuple(int(x) for x in args.pop(0).split(",")))
modes = [int(v) for v in args] or [1, 2]
for (N, d, BH) in shapes:
    g = torch.Generator(device="cuda").manual_seed(1)
    mk = lambda: fa_hip.jl_tensor(torch.randn((N, d, BH), generator=g, device="cuda"), torch.bfloat16)
    Q, K, V, dO = mk(), mk(), mk(), mk()
    Oo, l, m = fa_hip.dense_fa(Q, K, V)
    torch.cuda.synchronize()
    sl = lambda t: t[:, :, :1].float().cpu().double().numpy()
    ref = O.dense_fa_backward(sl(Q), sl(K), sl(V), sl(Oo), sl(dO), l[:, :, :1].cpu().double().numpy(),
                              m[:, :, :1].cpu().double().numpy())
    fl = 4.0 * BH * N * N * d * 2.5
    outs = {}
    for md in modes:
        L.fa_debug_set_bwd_mode(md)
        outs[md] = [x.clone() for x in fa_hip.dense_fa_backward(Q, K, V, Oo, dO, l, m)]
        torch.cuda.synchronize()
        errs = [float(np.abs(sl(x) - y).max() / np.abs(y).max()) for x, y in zip(outs[md], ref)]
        same = all(torch.equal(a, b) for a, b in zip(outs[md], outs[modes[0]]))
        print(f"N={N} d={d} BH={BH} mode {md}: rel err dQ/dK/dV {errs[0]:.2e} {errs[1]:.2e} {errs[2]:.2e}  "
              f"bitwise vs mode {modes[0]}: {same}", flush=True)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:
        fa_hip.dense_fa_backward(Q, K, V, Oo, dO, l, m)
        torch.cuda.synchronize()
    ts = {md: [] for md in modes}
    for rnd in range(5):
        for md in modes:
            L.fa_debug_set_bwd_mode(md)
            fa_hip.dense_fa_backward(Q, K, V, Oo, dO, l, m)
            e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3):
                fa_hip.dense_fa_backward(Q, K, V, Oo, dO, l, m)
            e1.record(); torch.cuda.synchronize()
            ts[md].append(e0.elapsed_time(e1) / 3 / 1e3)
    for md in modes:
        t = float(np.median(ts[md]))
        print(f"N={N} d={d} BH={BH} mode {md}: {t*1e3:.3f} ms  {fl/t/1e12:.1f} TFLOP/s (2.5x convention, "
              f"{fl/t/1e12/PEAK*100:.1f}% peak)  best {fl/min(ts[md])/1e12:.1f}", flush=True)
    L.fa_debug_set_bwd_mode(0)
