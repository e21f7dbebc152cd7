"""configs[2] as written (B = 1: 128x128 image, ws 7, d 64, bf16): device time per
call by HIP-graph replay for the windowed forward / backward kernel choices
(fa_debug_set_win_composed: 0 auto, 3 one-window row-shift, 6 two-window row-shift,
10 strip), after a clock settle.  Usage: python tools/exp/win_b1_modes.py [B]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import numpy as np, torch, fa_hip
from bench import time_graph, _randn_jl
L = fa_hip.lib()
B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
g = torch.Generator(device="cuda").manual_seed(1)
N, d, BH = 4096, 64, 64
Q, K, V = (_randn_jl(fa_hip, (N, d, BH), torch.bfloat16, g) for _ in range(3))
for _ in range(300):
    fa_hip.dense_fa(Q, K, V)
q, k, v, dy = (_randn_jl(fa_hip, (128, 128, 64, B), torch.bfloat16, g) for _ in range(4))
y0, l0, m0 = fa_hip.windowed_fa(q, k, v, 7)
g0 = fa_hip.windowed_fa_backward(q, k, v, y0, dy, l0, m0, 7)
for rnd in range(2):
    for mode in (0, 3, 6, 10):
        L.fa_debug_set_win_composed(mode)
        y, l, m = fa_hip.windowed_fa(q, k, v, 7)
        gr = fa_hip.windowed_fa_backward(q, k, v, y0, dy, l0, m0, 7)
        dy_ = float((y.float() - y0.float()).abs().max())
        dg = max(float((a.float() - b.float()).abs().max()) for a, b in zip(gr, g0))
        tf = time_graph(lambda: fa_hip.windowed_fa(q, k, v, 7), 50) * 1e6
        tb = time_graph(lambda: fa_hip.windowed_fa_backward(q, k, v, y0, dy, l0, m0, 7), 20) * 1e6
        print(f"B={B} mode {mode:2d}: fwd {tf:6.2f} us  bwd {tb:6.2f} us   max|dy| vs auto {dy_:.2e}  "
              f"max|dgrad| {dg:.2e}", flush=True)
L.fa_debug_set_win_composed(0)
