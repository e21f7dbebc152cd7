"""configs[2]-shaped windowed forward / backward in fp32 and f16 (device time, graph replay)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import torch, fa_hip
from bench import time_graph, _randn_jl
g = torch.Generator(device="cuda").manual_seed(1)
Q, K, V = (_randn_jl(fa_hip, (4096, 64, 64), torch.bfloat16, g) for _ in range(3))
for _ in range(200):
    fa_hip.dense_fa(Q, K, V)
for dt in (torch.float32, torch.float16, torch.bfloat16):
    for B in (1, 8):
        q, k, v, dy = (_randn_jl(fa_hip, (128, 128, 64, B), dt, g) for _ in range(4))
        y, lw, mw = fa_hip.windowed_fa(q, k, v, 7)
        tf = time_graph(lambda: fa_hip.windowed_fa(q, k, v, 7), 20)
        tb = time_graph(lambda: fa_hip.windowed_fa_backward(q, k, v, y, dy, lw, mw, 7), 10)
        print(f"{str(dt)[6:]:9s} B={B}: fwd {tf*1e6:8.1f} us  bwd {tb*1e6:8.1f} us", flush=True)
