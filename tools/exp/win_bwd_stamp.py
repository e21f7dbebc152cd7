"""Per-workgroup phase times of the fused windowed backward (win_bwd_rows) at
configs[2] geometry: s_memtime cycles per phase (median / p90 over workgroups)
and the realtime span.  Build first: python tools/exp/win_stamp.py build
Usage: python tools/exp/win_bwd_stamp.py [B...]"""
import ctypes, os, sys
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import numpy as np, torch, fa_hip
L = ctypes.CDLL(os.path.join(HERE, "libwin_stamp.so"))
P = lambda t: ctypes.c_void_p(t.data_ptr())
g = torch.Generator(device="cuda").manual_seed(1)
N, d, BH = 4096, 64, 64
Q, K, V = (fa_hip.jl_tensor(torch.randn((N, d, BH), device="cuda"), torch.bfloat16) for _ in range(3))
O = torch.empty_like(Q)
for B in [int(x) for x in (sys.argv[1:] or ["1", "16"])]:
    q, k, v, dy = (fa_hip.jl_tensor(torch.randn((128, 128, 64, B), generator=g, device="cuda"), torch.bfloat16)
                   for _ in range(4))
    y, lw, mw = fa_hip.windowed_fa(q, k, v, 7)
    dq, dk, dv = (torch.empty_like(q) for _ in range(3))
    out = np.zeros(8 * 361 * B, dtype=np.uint64)
    for rep in range(2):
        for _ in range(300):   # clock warm-up
            fa_hip.dense_fa_(O, fa_hip.jl_empty((N, 1, BH)), fa_hip.jl_empty((N, 1, BH)), Q, K, V)
        rc = L.stamp_run_bwd(P(q), P(k), P(v), P(y), P(dy), P(lw), P(mw), P(dq), P(dk), P(dv), B,
                             out.ctypes.data_as(ctypes.c_void_p))
        assert rc == 0, rc
        s = out.reshape(-1, 8).astype(np.int64)
        ph = np.diff(s[:, :5], axis=1)
        names = ["q/k loads + stage", "v/dy/y loads + stage + D", "phase 1 (S, dP, P, dS)", "phase 2 + stores"]
        print(f"B={B} rep {rep}: per-WG cycles (median/p90): " +
              ", ".join(f"{n}: {np.median(ph[:, i]):.0f}/{np.percentile(ph[:, i], 90):.0f}" for i, n in enumerate(names)))
        rt0, rt1 = s[:, 6], s[:, 7]
        print(f"   WG total median {np.median(s[:, 4] - s[:, 0]):.0f} cycles; realtime (100 MHz): WG span median "
              f"{np.median(rt1 - rt0):.0f}, first start -> last end {rt1.max() - rt0.min()}, "
              f"start spread {rt0.max() - rt0.min()}", flush=True)
