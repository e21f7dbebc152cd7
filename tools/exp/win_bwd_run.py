"""Run the configs[2]-shaped windowed backward (128x128x64 bf16, ws 7) a fixed
number of times at batch B — a workload for rocprofv3 --kernel-trace / --pmc
passes.  Usage: python tools/exp/win_bwd_run.py [B] [reps]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import torch, fa_hip
from bench import _randn_jl

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
g = torch.Generator(device="cuda").manual_seed(1)
q, k, v, dy = (_randn_jl(fa_hip, (128, 128, 64, B), torch.bfloat16, g) for _ in range(4))
y, lw, mw = fa_hip.windowed_fa(q, k, v, 7)
for _ in range(reps):
    fa_hip.windowed_fa(q, k, v, 7)
    fa_hip.windowed_fa_backward(q, k, v, y, dy, lw, mw, 7)
torch.cuda.synchronize()
print("ok", flush=True)
