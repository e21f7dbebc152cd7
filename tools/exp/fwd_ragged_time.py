"""Forward time on ragged shapes (Nk % 8 != 0 -> dense_fwd_generic) vs the
nearest aligned shape (fast path), HIP-graph replay after a warm-up."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import torch, fa_hip
from bench import time_graph, _randn_jl
g = torch.Generator(device="cuda").manual_seed(1)
for (N, d, B) in [(4096, 64, 64), (4095, 64, 64), (4097, 64, 64), (8192, 128, 16), (8191, 128, 16), (1000, 96, 16), (1001, 96, 16)]:
    Q, K, V = (_randn_jl(fa_hip, (N, d, B), torch.bfloat16, g) for _ in range(3))
    O = fa_hip.jl_empty((N, d, B), torch.bfloat16); l = fa_hip.jl_empty((N, 1, B)); m = fa_hip.jl_empty((N, 1, B))
    for _ in range(50):
        fa_hip.dense_fa_(O, l, m, Q, K, V)
    t = time_graph(lambda: fa_hip.dense_fa_(O, l, m, Q, K, V), 20)
    print(f"N={N} d={d} B={B}: {t*1e6:9.1f} us  {4.0*B*N*N*d/t/1e12:7.1f} TF", flush=True)
