"""A/B builds of libfa_hip.so on the configs[2]-shaped windowed BACKWARD (128x128x64
bf16, ws 7), B sweep, in ONE process: device time per call by HIP-graph replay after a
dense warm-up, rounds interleaved; gradients checked bitwise across the builds.
Usage: python tools/ab_lib_winbwd.py LIB_A LIB_B ... (env AB_B="1,8,32,128")"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import numpy as np, torch
import fa_hip
from bench import time_graph, _randn_jl

paths = sys.argv[1:]
libs = []
for p in paths:
    fa_hip._LIB = None
    os.environ["FA_HIP_LIB"] = os.path.abspath(p)
    libs.append(fa_hip.lib())
g = torch.Generator(device="cuda").manual_seed(1)
N, d, BH = 4096, 64, 64
Q, K, V = (_randn_jl(fa_hip, (N, d, BH), torch.bfloat16, g) for _ in range(3))
O = fa_hip.jl_empty((N, d, BH), torch.bfloat16)
l = fa_hip.jl_empty((N, 1, BH)); m = fa_hip.jl_empty((N, 1, BH))
fa_hip._LIB = libs[0]
for _ in range(400):
    fa_hip.dense_fa_(O, l, m, Q, K, V)
for B in [int(x) for x in os.environ.get("AB_B", "1,8,32,128").split(",")]:
    q, k, v, dy = (_randn_jl(fa_hip, (128, 128, 64, B), torch.bfloat16, g) for _ in range(4))
    y, lw, mw = fa_hip.windowed_fa(q, k, v, 7)
    nbytes = 7 * 128 * 128 * 64 * 2 * B     # q, k, v, dy read; dq, dk, dv written
    outs = []
    for L in libs:
        fa_hip._LIB = L
        outs.append([t.clone() for t in fa_hip.windowed_fa_backward(q, k, v, y, dy, lw, mw, 7)])
    torch.cuda.synchronize()
    for i in range(1, len(libs)):
        same = all(torch.equal(a, b) for a, b in zip(outs[0], outs[i]))
        print(f"B={B}: lib{i} vs lib0 bitwise equal={same}", flush=True)
    times = [[] for _ in libs]
    for rnd in range(5):
        for i, L in enumerate(libs):
            fa_hip._LIB = L
            for _ in range(20):
                fa_hip.dense_fa_(O, l, m, Q, K, V)
            times[i].append(time_graph(lambda: fa_hip.windowed_fa_backward(q, k, v, y, dy, lw, mw, 7), 50))
    for i, p in enumerate(paths):
        t = float(np.median(times[i]))
        print(f"B={B:3d} {os.path.basename(p):16s}: {t*1e6:8.2f} us  {nbytes/t/1e9:7.0f} GB/s (7-tensor count)", flush=True)
