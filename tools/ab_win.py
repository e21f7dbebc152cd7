"""configs[2] windowed forward: row-staged (0) vs register-gather (2) vs composed (1),
B sweep (GB/s of algorithmic traffic); outputs compared against the composed path."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import numpy as np, torch
import fa_hip
L = fa_hip.lib()
import ctypes
L.fa_debug_set_win_composed.argtypes = [ctypes.c_int]
for B in (1, 8, 32, 128):
    g = torch.Generator(device="cuda").manual_seed(1)
    q, k, v = (fa_hip.jl_tensor(torch.randn((128, 128, 64, B), generator=g, device="cuda"), torch.bfloat16) for _ in range(3))
    T, Lw = 49, 361
    alg = B * (4 * 128 * 128 * 64 * 2 + 2 * T * Lw * 4)
    res = {}
    for comp in (0, 2, 1):
        L.fa_debug_set_win_composed(comp)
        y, l, m = fa_hip.windowed_fa(q, k, v, 7)
        torch.cuda.synchronize()
        res[comp] = (y.float(), l.clone())
        ts = []
        for _ in range(5):
            e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10): fa_hip.windowed_fa(q, k, v, 7)
            e1.record(); torch.cuda.synchronize(); ts.append(e0.elapsed_time(e1) / 10 / 1e3)
        t = float(np.median(ts))
        name = {0: 'rows    ', 2: 'gather  ', 1: 'composed'}[comp]
        print(f"B={B:4d} {name}: {t*1e6:9.1f} us  {alg/t/1e9:8.1f} GB/s", flush=True)
    for c in (0, 2):
        dy = (res[c][0] - res[1][0]).abs().max()
        print(f"   {c} vs composed: max|dy| {float(dy):.3e}  max|dl| {float((res[c][1]-res[1][1]).abs().max()):.3e}")
    L.fa_debug_set_win_composed(0)
