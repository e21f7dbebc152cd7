"""Per-workgroup phase times of win_rows1 at configs[2] (B=1): s_memtime cycles
per phase (median over workgroups) and the realtime span of all workgroups.
Build first (CPU): python tools/exp/win_stamp.py build"""
import ctypes, os, subprocess, sys
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
ABL = int(os.environ.get("WABL", 0))   # FA_WIN_ABL of the stamped build (timing-only ablations)
SO = os.path.join(HERE, f"libwin_stamp{ABL or ''}.so")
if len(sys.argv) > 1 and sys.argv[1] == "build":
    B = os.path.join(ROOT, "flashattention.jl_amd", "csrc", "build")
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-shared",
                    "-fno-gpu-rdc", f"-DFA_WIN_ABL={ABL}", "-o", SO, "-x", "hip", os.path.join(HERE, "win_stamp.hip"),
                    "-x", "none", os.path.join(B, "fa_fwd.hip.o"), os.path.join(B, "fa_fwd_pers.hip.o"), os.path.join(B, "fa_fwd_p4.hip.o"), os.path.join(B, "fa_bwd.hip.o"),
                    os.path.join(B, "fa_f64.hip.o")], check=True)
    sys.exit(0)
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import numpy as np, torch, fa_hip
L = ctypes.CDLL(SO)
g = torch.Generator(device="cuda").manual_seed(1)
Bimg = int(os.environ.get("WB", 1))
q, k, v = (fa_hip.jl_tensor(torch.randn((128, 128, 64, Bimg), generator=g, device="cuda"), torch.bfloat16) for _ in range(3))
y = torch.empty_like(q)
l = torch.empty((49 * 361 * Bimg,), device="cuda"); m = torch.empty_like(l)
out = np.zeros(8 * 361 * Bimg, dtype=np.uint64)
P = lambda t: ctypes.c_void_p(t.data_ptr())
# warm the clock
N, d, BH = 4096, 64, 64
Q, K, V = (fa_hip.jl_tensor(torch.randn((N, d, BH), device="cuda"), torch.bfloat16) for _ in range(3))
O = torch.empty_like(Q); l2 = torch.empty((N * BH,), device="cuda"); m2 = torch.empty_like(l2)
for rep in range(3):
    for _ in range(300):
        fa_hip.dense_fa_(O, fa_hip.jl_empty((N, 1, BH)), fa_hip.jl_empty((N, 1, BH)), Q, K, V)
    rc = L.stamp_run(P(q), P(k), P(v), P(y), P(l), P(m), Bimg, out.ctypes.data_as(ctypes.c_void_p))
    assert rc == 0, rc
    nwg = (361 * Bimg + 1) // 2 if Bimg > 1 or os.environ.get("WPAIR") else 361 * Bimg
    s = out.reshape(-1, 8).astype(np.int64)[:nwg]
    s[:, 1] = s[:, 0]          # the row-shift kernel has no stamp 1 (no separate zero-fill phase)
    ph = np.diff(s[:, :6], axis=1)
    rt0, rt1 = s[:, 6], s[:, 7]
    names = ["-", "loads + stage + sync", "QK", "softmax", "PV + stores"]
    print(f"rep {rep}: per-WG phase cycles (median / p90): " +
          ", ".join(f"{n}: {np.median(ph[:, i]):.0f}/{np.percentile(ph[:, i], 90):.0f}" for i, n in enumerate(names)))
    print(f"   WG total cycles median {np.median(s[:, 5] - s[:, 0]):.0f}; realtime (100 MHz ticks): WG span median "
          f"{np.median(rt1 - rt0):.0f}, first start -> last end {rt1.max() - rt0.min()}, "
          f"start spread {rt0.max() - rt0.min()}; sum of WG spans / (kernel span x 768 slots) "
          f"{(rt1 - rt0).sum() / ((rt1.max() - rt0.min()) * 768):.2f}", flush=True)
    if rep == 2:
        span = np.percentile(rt1 - rt0, [10, 50, 90, 99])
        print("   WG realtime span percentiles 10/50/90/99 (10 ns ticks):", span, flush=True)
