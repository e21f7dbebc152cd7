"""configs[3] backward (8192, 128, 64 slabs) bf16, a fixed number of times in a given
mode (fa_debug_set_bwd_mode; 0 auto = single pass) — a workload for PMC passes.
Knobs (env): FA_L2LOCAL (-1 auto, 0, 1), FA_HOFF (chain step offset), FA_XCD (-1, 0),
FA_SHAPE "N,d,BH".
Usage: python tools/exp/bwd_run.py [mode] [reps]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import torch, fa_hip
mode = int(sys.argv[1]) if len(sys.argv) > 1 else 0
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
N, d, BH = (int(x) for x in os.environ.get("FA_SHAPE", "8192,128,64").split(","))
g = torch.Generator(device="cuda").manual_seed(1)
Q, K, V, dO = (fa_hip.jl_tensor(torch.randn((N, d, BH), generator=g, device="cuda"), torch.bfloat16) for _ in range(4))
O, l, m = fa_hip.dense_fa(Q, K, V)
L = fa_hip.lib()
L.fa_debug_set_bwd_mode(mode)
for k, f in (("FA_L2LOCAL", L.fa_debug_set_bwd_l2local), ("FA_HOFF", L.fa_debug_set_bwd_hoff),
             ("FA_XCD", L.fa_debug_set_bwd_xcd)):
    if k in os.environ:
        f(int(os.environ[k]))
for _ in range(reps):
    fa_hip.dense_fa_backward(Q, K, V, O, dO, l, m)
torch.cuda.synchronize()
print("ok status", fa_hip.backward_handoff_status(Q.device), flush=True)
