"""Circulant forward at (B*H=64, N=16384, d=64, W=129) bf16 x 10 — a workload for PMC passes."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import torch, fa_hip
g = torch.Generator(device="cuda").manual_seed(1)
Q, K, V = (fa_hip.jl_tensor(torch.randn((16384, 64, 64), generator=g, device="cuda"), torch.bfloat16) for _ in range(3))
for _ in range(10):
    fa_hip.circulant_fa(Q, K, V, 129)
torch.cuda.synchronize()
print("ok")
