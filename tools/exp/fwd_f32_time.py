"""fp32 forward (exact-f32 MFMA generic kernel) throughput vs the f32 MFMA peak."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import torch, fa_hip
from bench import time_graph
for (N, d, B) in [(4096, 64, 64), (2048, 128, 16), (512, 64, 4)]:
    Q, K, V = (fa_hip.jl_tensor(torch.randn((N, d, B), device="cuda"), torch.float32) for _ in range(3))
    O = fa_hip.jl_empty((N, d, B)); l = fa_hip.jl_empty((N, 1, B)); m = fa_hip.jl_empty((N, 1, B))
    for _ in range(20):
        fa_hip.dense_fa_(O, l, m, Q, K, V)
    t = time_graph(lambda: fa_hip.dense_fa_(O, l, m, Q, K, V), 10)
    print(f"fp32 fwd N={N} d={d} B={B}: {t*1e6:9.1f} us  {4.0*B*N*N*d/t/1e12:6.1f} TF (f32 MFMA peak 157)", flush=True)
