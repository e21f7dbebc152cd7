"""Per-window windowed backward, one vs two windows per workgroup (fa_debug_set_win_bwd_pair),
configs[2] geometry, B sweep, in one process: graph-replay device time per call after a
dense warm-up, rounds interleaved; gradients checked bitwise between the two forms.
Usage: python tools/exp/winbwd_pair_ab.py [B ...]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import numpy as np, torch
import fa_hip
from bench import time_graph, _randn_jl

L = fa_hip.lib()
g = torch.Generator(device="cuda").manual_seed(1)
N, d, BH = 4096, 64, 64
Q, K, V = (_randn_jl(fa_hip, (N, d, BH), torch.bfloat16, g) for _ in range(3))
O = fa_hip.jl_empty((N, d, BH), torch.bfloat16)
l = fa_hip.jl_empty((N, 1, BH)); m = fa_hip.jl_empty((N, 1, BH))
for _ in range(400):
    fa_hip.dense_fa_(O, l, m, Q, K, V)
for B in [int(x) for x in (sys.argv[1:] or ["1", "2", "4"])]:
    q, k, v, dy = (_randn_jl(fa_hip, (128, 128, 64, B), torch.bfloat16, g) for _ in range(4))
    y, lw, mw = fa_hip.windowed_fa(q, k, v, 7)
    outs = []
    for mode in (0, 1):
        L.fa_debug_set_win_bwd_pair(mode)
        outs.append([t.clone() for t in fa_hip.windowed_fa_backward(q, k, v, y, dy, lw, mw, 7)])
    torch.cuda.synchronize()
    same = all(torch.equal(a, b) for a, b in zip(*outs))
    times = {0: [], 1: []}
    for rnd in range(6):
        for mode in (0, 1):
            L.fa_debug_set_win_bwd_pair(mode)
            for _ in range(20):
                fa_hip.dense_fa_(O, l, m, Q, K, V)
            times[mode].append(time_graph(lambda: fa_hip.windowed_fa_backward(q, k, v, y, dy, lw, mw, 7), 50))
    L.fa_debug_set_win_bwd_pair(-1)
    print(f"B={B}: one window {np.median(times[0])*1e6:.2f} us, two windows {np.median(times[1])*1e6:.2f} us; "
          f"bitwise equal {same}", flush=True)
