"""Run forward variants at configs[1] (bf16, N=4096, d=64, B*H=64) a fixed number
of times each — a workload for rocprofv3 --pmc passes, where per-dispatch rows
are attributed by kernel name.  Usage: python tools/exp/fwd_run.py [variants...]"""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import torch
import fa_hip

L = fa_hip.lib()
variants = [int(v) for v in sys.argv[1:]] or [7, 8]
N, d, BH = int(os.environ.get("FA_N", 4096)), int(os.environ.get("FA_D", 64)), int(os.environ.get("FA_BH", 64))
g = torch.Generator(device="cuda").manual_seed(0)
Q, K, V = [fa_hip.jl_empty((N, d, BH), torch.bfloat16) for _ in range(3)]
for t in (Q, K, V):
    t.copy_(torch.randn((N, d, BH), generator=g, device="cuda"))
O = fa_hip.jl_empty((N, d, BH), torch.bfloat16)
l = fa_hip.jl_empty((N, 1, BH)); m = fa_hip.jl_empty((N, 1, BH))
for v in variants:
    L.fa_debug_set_fwd_variant(v)
    for _ in range(10):
        fa_hip.dense_fa_(O, l, m, Q, K, V)
    torch.cuda.synchronize()
L.fa_debug_set_fwd_variant(0)
print("ok")
