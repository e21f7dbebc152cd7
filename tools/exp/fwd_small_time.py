"""Forward on small grids (few workgroups): device time per call by graph replay."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import torch, fa_hip
from bench import time_graph, _randn_jl
g = torch.Generator(device="cuda").manual_seed(1)
Q, K, V = (_randn_jl(fa_hip, (4096, 64, 64), torch.bfloat16, g) for _ in range(3))
for _ in range(300):
    fa_hip.dense_fa(Q, K, V)
for (N, Nk, d, B, dt) in [(512, 512, 64, 4, torch.bfloat16), (512, 512, 64, 4, torch.float32), (4096, 4096, 64, 1, torch.bfloat16),
                          (16384, 16384, 64, 1, torch.bfloat16), (128, 32768, 128, 8, torch.bfloat16), (4096, 4096, 128, 4, torch.bfloat16)]:
    Qs = _randn_jl(fa_hip, (N, d, B), dt, g); Ks = _randn_jl(fa_hip, (Nk, d, B), dt, g); Vs = _randn_jl(fa_hip, (Nk, d, B), dt, g)
    O = fa_hip.jl_empty((N, d, B), dt); l = fa_hip.jl_empty((N, 1, B)); m = fa_hip.jl_empty((N, 1, B))
    t = time_graph(lambda: fa_hip.dense_fa_(O, l, m, Qs, Ks, Vs), 20)
    print(f"N={N} Nk={Nk} d={d} B={B} {str(dt)[6:]}: {t*1e6:9.1f} us  {4.0*B*N*Nk*d/t/1e12:7.1f} TF", flush=True)
