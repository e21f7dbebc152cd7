"""A/B: configs[1] forward issued as K stream launches vs one HIP graph of K
launches (same kernels), alternating, after a settle.  Device time per step from
events; also wall time per step."""
import os, sys, time, json, statistics
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import torch
import bench, fa_hip

N, D, BH, K = 4096, 64, 64, 20
gen = torch.Generator(device="cuda").manual_seed(1)
Q, Kt, V = (bench._randn_jl(fa_hip, (N, D, BH), torch.bfloat16, gen) for _ in range(3))
O = fa_hip.jl_empty((N, D, BH), torch.bfloat16)
l = fa_hip.jl_empty((N, 1, BH)); m = fa_hip.jl_empty((N, 1, BH))
step = lambda: fa_hip.dense_fa_(O, l, m, Q, Kt, V)
side = torch.cuda.Stream()
side.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(side):
    step(); step()
torch.cuda.current_stream().wait_stream(side)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    for _ in range(K):
        step()
torch.cuda.synchronize()
bench.settle(step, 0.4)
flops = 4.0 * BH * N * N * D
res = {"stream": [], "graph": []}
for rep in range(6):
    for name, fn in (("stream", lambda: [step() for _ in range(K)]), ("graph", g.replay)):
        fn(); torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter(); e0.record(); fn(); e1.record(); torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        res[name].append((e0.elapsed_time(e1) / K, wall * 1e3 / K))
for name, xs in res.items():
    ev = statistics.median(x[0] for x in xs); wl = statistics.median(x[1] for x in xs)
    print(f"{name:6s}: event {ev * 1e3:7.1f} us/step ({flops / ev / 1e9:7.1f} TFLOP/s), wall {wl * 1e3:7.1f} us/step ({flops / wl / 1e9:7.1f} TFLOP/s)")
