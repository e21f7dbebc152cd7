"""Timing-only ablations of win_rows1s at configs[2] (128x128, ws 7, d 64), B=32:
0 = product, 1 = no y stores, 2 = all row loads from one address, 3 = both.
Build (CPU): python tools/exp/win_ablate.py build; run on the GPU without args."""
import ctypes, os, subprocess, sys
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
MODES = (0, 1, 2, 3)
so = lambda a: os.path.join(HERE, f"libwin_abl{a}.so")
if len(sys.argv) > 1 and sys.argv[1] == "build":
    B = os.path.join(ROOT, "flashattention.jl_amd", "csrc", "build")
    for a in MODES:
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-shared",
                        "-fno-gpu-rdc", f"-DFA_WIN_ABL={a}", "-o", so(a), "-x", "hip", os.path.join(HERE, "win_ablate.hip"),
                        "-x", "none", os.path.join(B, "fa_fwd.hip.o"), os.path.join(B, "fa_bwd.hip.o")], check=True)
    sys.exit(0)
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import numpy as np, torch, fa_hip
Bimg = int(os.environ.get("WB", 32))
g = torch.Generator(device="cuda").manual_seed(1)
q, k, v = (fa_hip.jl_tensor(torch.randn((128, 128, 64, Bimg), generator=g, device="cuda"), torch.bfloat16) for _ in range(3))
y = torch.empty_like(q)
l = torch.empty((49 * 361 * Bimg,), device="cuda"); m = torch.empty_like(l)
P = lambda t: ctypes.c_void_p(t.data_ptr())
libs = {a: ctypes.CDLL(so(a)) for a in MODES}
N, d, BH = 4096, 64, 64
Q, K, V = (fa_hip.jl_tensor(torch.randn((N, d, BH), device="cuda"), torch.bfloat16) for _ in range(3))
O = torch.empty_like(Q)
for _ in range(200):
    fa_hip.dense_fa_(O, fa_hip.jl_empty((N, 1, BH)), fa_hip.jl_empty((N, 1, BH)), Q, K, V)
ts = {a: [] for a in MODES}
for rnd in range(7):
    for a in MODES:
        f = libs[a].abl_run
        f(P(q), P(k), P(v), P(y), P(l), P(m), Bimg)
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            f(P(q), P(k), P(v), P(y), P(l), P(m), Bimg)
        e1.record(); torch.cuda.synchronize()
        ts[a].append(e0.elapsed_time(e1) / 20 * 1e3)
byt = Bimg * (4 * 128 * 128 * 64 * 2 + 2 * 49 * 361 * 4)
for a in MODES:
    t = float(np.median(ts[a]))
    print(f"B={Bimg} ablation {a}: {t:.1f} us  ({byt / t / 1e3:.0f} GB/s algorithmic)", flush=True)
