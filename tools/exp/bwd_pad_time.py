"""Backward time on shapes outside the MFMA kernels' set: padded fast path
(default) vs the generic SIMT path (fa_debug_set_bwd_generic(1)), HIP-graph replay."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import torch, fa_hip
from bench import time_graph, _randn_jl
L = fa_hip.lib()
g = torch.Generator(device="cuda").manual_seed(1)
for (N, d, dv, B) in [(4095, 64, 64, 64), (1000, 96, 96, 16), (30, 12, 6, 2), (8191, 128, 128, 8)]:
    Q, K = (_randn_jl(fa_hip, (N, d, B), torch.bfloat16, g) for _ in range(2))
    V, dO = (_randn_jl(fa_hip, (N, dv, B), torch.bfloat16, g) for _ in range(2))
    O, l, m = fa_hip.dense_fa(Q, K, V)
    fl = 10.0 * B * N * N * (d + dv) / 2
    res = []
    for gen in (0, 1):
        L.fa_debug_set_bwd_generic(gen)
        steps = 3 if gen else 10
        t = time_graph(lambda: fa_hip.dense_fa_backward(Q, K, V, O, dO, l, m), steps)
        res.append(t)
    L.fa_debug_set_bwd_generic(0)
    print(f"N={N} d={d} dv={dv} B={B}: padded-fast {res[0]*1e6:9.1f} us ({fl/res[0]/1e12:6.1f} TF)  "
          f"generic {res[1]*1e6:9.1f} us  x{res[1]/res[0]:.1f}", flush=True)
q, k, v, dy = (_randn_jl(fa_hip, (128, 128, 64, 1), torch.bfloat16, g) for _ in range(4))
y, lw, mw = fa_hip.windowed_fa(q, k, v, 7, stride=4)
t = time_graph(lambda: fa_hip.windowed_fa_backward(q, k, v, y, dy, lw, mw, 7, stride=4), 10)
print(f"windowed backward 128x128x64 ws 7 stride 4 (overlapping, composed): {t*1e6:.1f} us", flush=True)
for (N, d, B) in [(4096, 64, 64), (512, 64, 4), (2048, 128, 16)]:
    Q, K, V, dO = (fa_hip.jl_tensor(torch.randn((N, d, B), device="cuda"), torch.float32) for _ in range(4))
    O, l, m = fa_hip.dense_fa(Q, K, V)
    res = []
    for gen in (0, 1):
        L.fa_debug_set_bwd_generic(gen)
        res.append(time_graph(lambda: fa_hip.dense_fa_backward(Q, K, V, O, dO, l, m), 3))
    L.fa_debug_set_bwd_generic(0)
    fl = 10.0 * B * N * N * d
    print(f"fp32 N={N} d={d} B={B}: mfma {res[0]*1e6:9.1f} us ({fl/res[0]/1e12:6.1f} TF)  generic {res[1]*1e6:9.1f} us  x{res[1]/res[0]:.1f}", flush=True)
