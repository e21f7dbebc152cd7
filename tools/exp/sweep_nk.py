"""Fixed (prologue/epilogue) vs per-tile cost: time the forward at N=4096 for several Nk."""
import ctypes, os, sys
import numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import fa_hip
L = fa_hip.lib()
var = int(sys.argv[1]) if len(sys.argv) > 1 else 1
L.fa_debug_set_fwd_variant(var)
N, d, BH = 4096, 64, 64
for Nk in (64, 256, 1024, 2048, 4096, 8192):
    g = torch.Generator(device="cuda").manual_seed(1)
    Q = fa_hip.jl_empty((N, d, BH), torch.bfloat16); Q.copy_(torch.randn((N, d, BH), generator=g, device="cuda"))
    K = fa_hip.jl_empty((Nk, d, BH), torch.bfloat16); K.copy_(torch.randn((Nk, d, BH), generator=g, device="cuda"))
    V = fa_hip.jl_empty((Nk, d, BH), torch.bfloat16); V.copy_(torch.randn((Nk, d, BH), generator=g, device="cuda"))
    O = fa_hip.jl_empty((N, d, BH), torch.bfloat16); l = fa_hip.jl_empty((N, 1, BH)); m = fa_hip.jl_empty((N, 1, BH))
    for _ in range(3): fa_hip.dense_fa_(O, l, m, Q, K, V)
    ts = []
    for _ in range(5):
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10): fa_hip.dense_fa_(O, l, m, Q, K, V)
        e1.record(); torch.cuda.synchronize(); ts.append(e0.elapsed_time(e1) / 10)
    t = np.median(ts)
    print(f"Nk={Nk:5d}  {t*1e3:8.1f} us  {4.0*BH*N*Nk*d/(t/1e3)/1e12:7.1f} TF", flush=True)
