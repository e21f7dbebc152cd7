"""configs[3] backward (4,16,8192,128) bf16 x 5 after a warm-up — a workload for rocprofv3."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import torch, fa_hip
from bench import _randn_jl
g = torch.Generator(device="cuda").manual_seed(1)
N, d, BH = int(os.environ.get("FA_N", 8192)), int(os.environ.get("FA_D", 128)), 64
Q, K, V, dO = (_randn_jl(fa_hip, (N, d, BH), torch.bfloat16, g) for _ in range(4))
O, l, m = fa_hip.dense_fa(Q, K, V)
for _ in range(int(os.environ.get("FA_REPS", 8))):
    fa_hip.dense_fa_backward(Q, K, V, O, dO, l, m)
torch.cuda.synchronize()
print("ok")
