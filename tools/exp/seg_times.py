"""TEMP: per-segment s_memtime breakdown of the ping-pong forward (FA_ABLATE bit 8).
Usage: FA_ABLATE=8 python tools/exp/seg_times.py <variant>"""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import numpy as np, torch
import fa_hip
L = fa_hip.lib()
v = int(sys.argv[1]) if len(sys.argv) > 1 else 8
N, d, BH = 4096, 64, 64
g = torch.Generator(device="cuda").manual_seed(0)
Q, K, V = [fa_hip.jl_empty((N, d, BH), torch.bfloat16) for _ in range(3)]
for t in (Q, K, V): t.copy_(torch.randn((N, d, BH), generator=g, device="cuda"))
O = fa_hip.jl_empty((N, d, BH), torch.bfloat16)
l = fa_hip.jl_empty((N, 1, BH)); m = fa_hip.jl_empty((N, 1, BH))
L.fa_debug_set_fwd_variant(v)
for _ in range(3): fa_hip.dense_fa_(O, l, m, Q, K, V)
O.zero_(); fa_hip.dense_fa_(O, l, m, Q, K, V); torch.cuda.synchronize()
nwg = 64 * ((N + 255) // 256)
ts = O.permute(2, 1, 0).contiguous().view(torch.int64).flatten()[: nwg * 8 * 20].cpu().numpy().reshape(nwg, 8, 4, 5).astype(np.float64)
M = ts[..., 1] - ts[..., 0]; BM = ts[..., 2] - ts[..., 1]; Vs = ts[..., 3] - ts[..., 2]; BV = ts[..., 4] - ts[..., 3]
tot = ts[..., 4] - ts[..., 0]
for name, x in [("M seg", M), ("barrier after M", BM), ("V seg", Vs), ("barrier after V", BV), ("tile total", tot)]:
    a = x[:, :4].flatten(); b = x[:, 4:].flatten()
    print(f"{name:18s} grpA med {np.median(a):7.0f} p90 {np.percentile(a,90):7.0f} | grpB med {np.median(b):7.0f} p90 {np.percentile(b,90):7.0f}")
