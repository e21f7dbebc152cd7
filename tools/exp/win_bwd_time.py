"""configs[2]-shaped windowed backward (128x128x64 bf16, ws 7): device time per
call by HIP-graph replay, B sweep, next to the forward.  Usage: python tools/exp/win_bwd_time.py"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import torch, fa_hip
from bench import time_graph, _randn_jl
g = torch.Generator(device="cuda").manual_seed(1)
N, d, BH = 4096, 64, 64
Q, K, V = (_randn_jl(fa_hip, (N, d, BH), torch.bfloat16, g) for _ in range(3))
O = fa_hip.jl_empty((N, d, BH), torch.bfloat16); l = fa_hip.jl_empty((N, 1, BH)); m = fa_hip.jl_empty((N, 1, BH))
for _ in range(400):
    fa_hip.dense_fa_(O, l, m, Q, K, V)
for B in [int(x) for x in (sys.argv[1:] or ["1", "8", "32"])]:
    q, k, v, dy = (_randn_jl(fa_hip, (128, 128, 64, B), torch.bfloat16, g) for _ in range(4))
    y, lw, mw = fa_hip.windowed_fa(q, k, v, 7)
    tf = time_graph(lambda: fa_hip.windowed_fa(q, k, v, 7), 50)
    tb = time_graph(lambda: fa_hip.windowed_fa_backward(q, k, v, y, dy, lw, mw, 7), 20)
    # algorithmic bytes of the backward: q, k, v, dy read, dq, dk, dv written (bf16) + l, m (y not needed)
    byt = B * (7 * 128 * 128 * 64 * 2 + 2 * 49 * 361 * 4)
    print(f"B={B:3d}: fwd {tf*1e6:8.1f} us   bwd {tb*1e6:8.1f} us  ({byt/tb/1e9:6.0f} GB/s algorithmic)", flush=True)
