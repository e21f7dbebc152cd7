"""Time the backward (fast vs generic) on configs[3] and check against the oracle on one slab."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import numpy as np, torch
import fa_hip
from oracle import fa_oracle as O
L = fa_hip.lib()
PEAK = 2516.58
for (N, d, BH) in [(8192, 128, 64), (4096, 64, 64)]:
    g = torch.Generator(device="cuda").manual_seed(1)
    mk = lambda: fa_hip.jl_tensor(torch.randn((N, d, BH), generator=g, device="cuda"), torch.bfloat16)
    Q, K, V, dO = mk(), mk(), mk(), mk()
    Oo, l, m = fa_hip.dense_fa(Q, K, V)
    torch.cuda.synchronize()
    sl = lambda t: t[:, :, :1].float().cpu().double().numpy()
    ref = O.dense_fa_backward(sl(Q), sl(K), sl(V), sl(Oo), sl(dO), l[:, :, :1].cpu().double().numpy(), m[:, :, :1].cpu().double().numpy())
    fl = 4.0 * BH * N * N * d * 2.5
    for gen in (0, 1):
        if gen and N * d > 4096 * 64: continue
        L.fa_debug_set_bwd_generic(gen)
        dQ, dK, dV = fa_hip.dense_fa_backward(Q, K, V, Oo, dO, l, m)
        torch.cuda.synchronize()
        errs = [float(np.abs(sl(x) - y).max() / np.abs(y).max()) for x, y in zip((dQ, dK, dV), ref)]
        ts = []
        for _ in range(3):
            e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3): fa_hip.dense_fa_backward(Q, K, V, Oo, dO, l, m)
            e1.record(); torch.cuda.synchronize(); ts.append(e0.elapsed_time(e1) / 3 / 1e3)
        t = float(np.median(ts))
        print(f"N={N} d={d} {'generic' if gen else 'fast'}: {t*1e3:.2f} ms  {fl/t/1e12:.1f} TFLOP/s ({fl/t/1e12/PEAK*100:.1f}%)  rel err dQ/dK/dV {errs[0]:.2e} {errs[1]:.2e} {errs[2]:.2e}", flush=True)
    L.fa_debug_set_bwd_generic(0)
