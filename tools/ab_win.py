"""configs[2] windowed forward, B sweep: auto (0) vs one-window row-shift (3) vs
two-window row-shift (6) vs four-window row-scatter (4) vs register-gather (2).
Device time per call from HIP-graph replay (bench.time_graph), GB/s of algorithmic
traffic; outputs compared against the four-window path."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import torch
import fa_hip
from bench import time_graph
L = fa_hip.lib()
L.fa_debug_set_win_composed.argtypes = [ctypes.c_int]
NAMES = {0: "auto    ", 3: "rows1   ", 6: "rows1x2 ", 4: "rows4   ", 2: "gather  ", 1: "composed",
         10: "strip8  ", 12: "rows1x3 "}
MODES = [int(x) for x in os.environ.get("WMODES", "0,3,6,4,2").split(",")]
Bs = [int(x) for x in sys.argv[1:]] or [1, 2, 4, 8, 32, 128]
for B in Bs:
    g = torch.Generator(device="cuda").manual_seed(1)
    q, k, v = (fa_hip.jl_tensor(torch.randn((128, 128, 64, B), generator=g, device="cuda"), torch.bfloat16) for _ in range(3))
    T, Lw = 49, 361
    alg = B * (4 * 128 * 128 * 64 * 2 + 2 * T * Lw * 4)
    res, ts = {}, {c: [] for c in MODES}
    for comp in MODES:
        L.fa_debug_set_win_composed(comp)
        y, l, m = fa_hip.windowed_fa(q, k, v, 7)
        torch.cuda.synchronize()
        res[comp] = (y.float(), l.clone())
    for rnd in range(int(os.environ.get("WROUNDS", 1))):   # interleaved rounds, median reported
        for comp in MODES:
            L.fa_debug_set_win_composed(comp)
            ts[comp].append(time_graph(lambda: fa_hip.windowed_fa(q, k, v, 7), 20))
    for comp in MODES:
        t = sorted(ts[comp])[len(ts[comp]) // 2]
        print(f"B={B:4d} {NAMES[comp]}: {t*1e6:9.2f} us  {alg/t/1e9:8.1f} GB/s  (min {min(ts[comp])*1e6:.2f})", flush=True)
    ref = MODES[-1]
    for c in MODES[:-1]:
        dy = (res[c][0] - res[ref][0]).abs().max()
        print(f"   {c} vs {ref}: max|dy| {float(dy):.3e}  max|dl| {float((res[c][1]-res[ref][1]).abs().max()):.3e}")
    L.fa_debug_set_win_composed(0)
