"""Phase stamps of the single-pass backward (a -DFA_BWD_STAMP4=w build): median cycles
per phase over steps 8..119 of workgroup w at configs[3], for 8 and 4 waves.
Usage: FA_HIP_LIB=stamped.so python tools/exp/bwd4_stamp.py"""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import numpy as np, torch, fa_hip
N, d, BH = 8192, 128, 64
g = torch.Generator(device="cuda").manual_seed(1)
mk = lambda: fa_hip.jl_tensor(torch.randn((N, d, BH), generator=g, device="cuda"), torch.bfloat16)
Q, K, V, dO = mk(), mk(), mk(), mk()
O, l, m = fa_hip.dense_fa(Q, K, V)
L = fa_hip.lib()
if os.environ.get("FA_BWD_MODE"):   # timing-only ablations of a -DFA_BWD_ABL build (WRONG dQ)
    assert L.fa_debug_set_bwd_mode(int(os.environ["FA_BWD_MODE"])) >= 0
buf = (ctypes.c_ulonglong * (128 * 16))()
names = {0: "B1", 1: "SdP0", 2: "SdP1|V0", 3: "A0", 4: "SdP2|V1", 5: "A1", 6: "SdP3|V2", 7: "A2|V3", 8: "A3/phaseA",
         9: "B2", 10: "dQ"}
for w in ((8, 4) if hasattr(L, "fa_debug_set_bwd_waves") else (8,)):
    if w != 8:
        L.fa_debug_set_bwd_waves(w)
    for _ in range(3):
        fa_hip.dense_fa_backward(Q, K, V, O, dO, l, m)
    torch.cuda.synchronize()
    assert L.fa_debug_bwd_stamps(buf, 128 * 16) == 0
    a = np.array(buf, dtype=np.int64).reshape(128, 16)
    pts = [0, 8, 9, 10] if w == 8 else list(range(11))
    print(f"waves={w}: per-step cycles (median over steps 8..119)")
    step = np.median(a[9:120, 0] - a[8:119, 0])
    print(f"  step {step:.0f}")
    for k0, k1 in zip(pts, pts[1:]):
        print(f"  {names[k0]:>10s} -> {names[k1]:<10s} {np.median(a[8:120, k1] - a[8:120, k0]):8.0f}")
    print(f"  {'dQ':>10s} -> next B1    {np.median(a[9:120, 0] - a[8:119, 10]):8.0f}", flush=True)
