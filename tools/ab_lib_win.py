"""A/B builds of libfa_hip.so on the configs[2] windowed forward (128x128x64 bf16,
ws 7), B sweep, in ONE process: device time per call by HIP-graph replay after a
dense warm-up, rounds interleaved across libraries.
Usage: python tools/ab_lib_win.py LIB_A LIB_B ... (env AB_B="1,2,4,8,32")"""
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
for B in [int(x) for x in os.environ.get("AB_B", "1,2,4,8,32").split(",")]:
    q, k, v = (_randn_jl(fa_hip, (128, 128, 64, B), torch.bfloat16, g) for _ in range(3))
    alg = B * (4 * 128 * 128 * 64 * 2 + 2 * 49 * 361 * 4)
    outs = []
    for L in libs:
        fa_hip._LIB = L
        outs.append(fa_hip.windowed_fa(q, k, v, 7)[0].float())
    torch.cuda.synchronize()
    for i in range(1, len(libs)):
        print(f"B={B}: lib{i} vs lib0 bitwise equal={bool(torch.equal(outs[0], outs[i]))}", flush=True)
    times = [[] for _ in libs]
    for rnd in range(5):
        for i, L in enumerate(libs):
            fa_hip._LIB = L
            for _ in range(20):
                fa_hip.dense_fa_(O, l, m, Q, K, V)
            times[i].append(time_graph(lambda: fa_hip.windowed_fa(q, k, v, 7), 100))
    for i, p in enumerate(paths):
        t = float(np.median(times[i]))
        print(f"B={B:3d} {os.path.basename(p):14s}: {t*1e6:8.2f} us  {alg/t/1e9:7.0f} GB/s", flush=True)
