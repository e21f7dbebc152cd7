"""configs[2] windowed forward (128x128x64 bf16, ws 7, B images) x 10 — a workload for PMC passes."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import torch, fa_hip
B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
fa_hip.lib().fa_debug_set_win_composed(int(os.environ.get("WMODE", 0)))   # 6 = register-staged two-window
g = torch.Generator(device="cuda").manual_seed(1)
q, k, v = (fa_hip.jl_tensor(torch.randn((128, 128, 64, B), generator=g, device="cuda"), torch.bfloat16) for _ in range(3))
for _ in range(10):
    fa_hip.windowed_fa(q, k, v, 7)
torch.cuda.synchronize()
print("ok")
