"""A/B the forward kernel variants in ONE process (interleaved rounds) on
configs[1] and configs[3]-fwd; checks each variant against the oracle on one
slab.  Usage: python tools/ab_fwd.py [variants...]"""
import ctypes, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import numpy as np, torch
import fa_hip
from oracle import fa_oracle as O

L = fa_hip.lib()
L.fa_debug_set_fwd_variant.restype = ctypes.c_int
variants = [int(v) for v in sys.argv[1:]] or [0, 4, 5, 6, 7]
PEAK = 2516.58

def mk(N, d, BH, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    out = []
    for _ in range(3):
        t = fa_hip.jl_empty((N, d, BH), torch.bfloat16)
        t.copy_(torch.randn((N, d, BH), generator=g, device="cuda"))
        out.append(t)
    return out

for (N, d, BH) in [(4096, 64, 64), (8192, 128, 64)]:
    Q, K, V = mk(N, d, BH, 1)
    O_ = fa_hip.jl_empty((N, d, BH), torch.bfloat16)
    l = fa_hip.jl_empty((N, 1, BH)); m = fa_hip.jl_empty((N, 1, BH))
    flops = 4.0 * BH * N * N * d
    ref = O.dense_fa3(Q[:, :, :1].float().cpu().double().numpy(), K[:, :, :1].float().cpu().double().numpy(),
                      V[:, :, :1].float().cpu().double().numpy())
    times = {v: [] for v in variants}
    for v in variants:
        L.fa_debug_set_fwd_variant(v)
        fa_hip.dense_fa_(O_, l, m, Q, K, V)
        torch.cuda.synchronize()
        err = np.abs(O_[:, :, :1].float().cpu().numpy() - ref[0]).max()
        lerr = np.abs(l[:, :, :1].cpu().numpy() - ref[1]).max() / ref[1].max()
        merr = np.abs(m[:, :, :1].cpu().numpy() - ref[2]).max()
        print(f"N={N} d={d} variant {v}: max|dO|={err:.3e} rel|dl|={lerr:.2e} |dm|={merr:.2e}", flush=True)
    for rnd in range(6):
        for v in variants:
            L.fa_debug_set_fwd_variant(v)
            for _ in range(2):
                fa_hip.dense_fa_(O_, l, m, Q, K, V)
            e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                fa_hip.dense_fa_(O_, l, m, Q, K, V)
            e1.record(); torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1) / 10 / 1e3)
    for v in variants:
        t = np.median(times[v])
        print(f"N={N} d={d} variant {v}: {t*1e6:.1f} us  {flops/t/1e12:.1f} TFLOP/s  ({flops/t/1e12/PEAK*100:.1f}% peak)  min {flops/min(times[v])/1e12:.1f}", flush=True)
    L.fa_debug_set_fwd_variant(0)
