"""Circulant forward across dtypes / ragged N (device time, graph replay)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import torch, fa_hip
from bench import time_graph, _randn_jl
g = torch.Generator(device="cuda").manual_seed(1)
Q, K, V = (_randn_jl(fa_hip, (4096, 64, 64), torch.bfloat16, g) for _ in range(3))
for _ in range(200):
    fa_hip.dense_fa(Q, K, V)
for (N, d, B, W, dt) in [(16384, 64, 64, 129, torch.bfloat16), (16383, 64, 64, 129, torch.bfloat16),
                         (16384, 64, 64, 129, torch.float32), (4096, 32, 1, 129, torch.float32)]:
    Qc, Kc, Vc = (_randn_jl(fa_hip, (N, d, B), dt, g) for _ in range(3))
    Oc = fa_hip.jl_empty((N, d, B), dt); lc = fa_hip.jl_empty((N, 1, B)); mc = fa_hip.jl_empty((N, 1, B))
    t = time_graph(lambda: fa_hip.circulant_fa_(Oc, lc, mc, Qc, Kc, Vc, W), 10)
    esz = 4 if dt == torch.float32 else 2
    print(f"circ N={N} d={d} B={B} W={W} {str(dt)[6:]}: {t*1e6:9.1f} us  {B*N*(4*d*esz+8)/t/1e9:7.0f} GB/s", flush=True)
