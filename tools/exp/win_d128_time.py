"""Windowed forward/backward with d = 128 (composed path) at 128x128, ws 7 (graph replay)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import torch, fa_hip
from bench import time_graph, _randn_jl
g = torch.Generator(device="cuda").manual_seed(1)
for B in (1, 8):
    q, k, v, dy = (_randn_jl(fa_hip, (128, 128, 128, B), torch.bfloat16, g) for _ in range(4))
    y, lw, mw = fa_hip.windowed_fa(q, k, v, 7)
    tf = time_graph(lambda: fa_hip.windowed_fa(q, k, v, 7), 10)
    tb = time_graph(lambda: fa_hip.windowed_fa_backward(q, k, v, y, dy, lw, mw, 7), 5)
    print(f"d=128 B={B}: fwd {tf*1e6:8.1f} us  bwd {tb*1e6:8.1f} us", flush=True)
