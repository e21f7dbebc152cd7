"""configs[2] windowed forward at small batch: device time per call by HIP-graph
replay on a warm GPU (400 dense launches first), beside the per-node floor of a
1-element torch kernel in the same kind of graph.  Usage: python tools/exp/win_latency.py"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import torch, fa_hip
import bench

g = torch.Generator(device="cuda").manual_seed(1)
N, d, BH = 4096, 64, 64
Q, K, V = (bench._randn_jl(fa_hip, (N, d, BH), torch.bfloat16, g) for _ in range(3))
O = fa_hip.jl_empty((N, d, BH), torch.bfloat16)
l = fa_hip.jl_empty((N, 1, BH)); m = fa_hip.jl_empty((N, 1, BH))
for _ in range(400):
    fa_hip.dense_fa_(O, l, m, Q, K, V)
torch.cuda.synchronize()
x = torch.zeros(1, device="cuda")
print(f"1-element add_: {bench.time_graph(lambda: x.add_(1.0), 200) * 1e6:.2f} us per node", flush=True)
for B in (1, 2, 4, 8, 32):
    q, k, v = (bench._randn_jl(fa_hip, (128, 128, 64, B), torch.bfloat16, g) for _ in range(3))
    for _ in range(100):
        fa_hip.dense_fa_(O, l, m, Q, K, V)
    t = bench.time_graph(lambda: fa_hip.windowed_fa(q, k, v, 7), 200)
    byt = B * (4 * 128 * 128 * 64 * 2 + 2 * 49 * 361 * 4)
    print(f"windowed B={B}: {t*1e6:.2f} us  {byt/t/1e9:.0f} GB/s", flush=True)
