"""Per-launch time series of the configs[1] forward from a cold start: shows
how many launches the GPU needs to reach its sustained clock (sizes bench.py's
default warm-up).  Usage: python tools/exp/ramp.py [launches]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import numpy as np, torch
import fa_hip

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4000
N, d, BH = 4096, 64, 64
g = torch.Generator(device="cuda").manual_seed(0)
Q, K, V = [fa_hip.jl_empty((N, d, BH), torch.bfloat16) for _ in range(3)]
for t in (Q, K, V):
    t.copy_(torch.randn((N, d, BH), generator=g, device="cuda"))
O = fa_hip.jl_empty((N, d, BH), torch.bfloat16)
l = fa_hip.jl_empty((N, 1, BH)); m = fa_hip.jl_empty((N, 1, BH))
torch.cuda.synchronize()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]
ev[0].record()
for i in range(n):
    fa_hip.dense_fa_(O, l, m, Q, K, V)
    ev[i + 1].record()
torch.cuda.synchronize()
t = np.array([ev[i].elapsed_time(ev[i + 1]) * 1e3 for i in range(n)])
for a, b in [(0, 10), (10, 20), (20, 50), (50, 70), (70, 100), (100, 200), (200, 500), (500, 1000),
             (1000, 2000), (2000, 3000), (3000, n)]:
    if b <= n:
        print(f"launches {a:5d}-{b:5d}: median {np.median(t[a:b]):7.1f} us  mean {t[a:b].mean():7.1f}", flush=True)
