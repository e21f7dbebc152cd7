"""configs[1] forward (4096, 64, 64) bf16: 300 launches of the default 8-wave kernel
(w8q2_wide) and 300 of the persistent variant 40 (fa_fwd_pers.hip), interleaved in
blocks of 50 after a settle, for a rocprofv3 --kernel-trace --stats comparison."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import torch, fa_hip
L = fa_hip.lib()
L.fa_debug_fwd_last_path.restype = ctypes.c_int
g = torch.Generator(device="cuda").manual_seed(1)
N, d, BH = 4096, 64, 64
Q, K, V = (fa_hip.jl_tensor(torch.randn((N, d, BH), generator=g, device="cuda"), torch.bfloat16) for _ in range(3))
O = fa_hip.jl_empty((N, d, BH), torch.bfloat16)
l = fa_hip.jl_empty((N, 1, BH)); m = fa_hip.jl_empty((N, 1, BH))
for _ in range(600):
    fa_hip.dense_fa_(O, l, m, Q, K, V)
paths = {}
for blk in range(6):
    for v in (0, 40):
        old = L.fa_debug_set_fwd_variant(v)
        for _ in range(50):
            fa_hip.dense_fa_(O, l, m, Q, K, V)
        torch.cuda.synchronize()
        paths[v] = L.fa_debug_fwd_last_path()
        L.fa_debug_set_fwd_variant(old)
print("last paths:", paths)
