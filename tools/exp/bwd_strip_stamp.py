"""Per-workgroup phase cycles of the strip windowed backward (win_bwd_strip, mode 10)
at configs[2] (128x128, ws 7, d 64, bf16), B = 32 by default: s_memtime cycles per
phase (median / p90 over workgroups), the in-kernel clock, the workgroup realtime
span, and how many workgroups ran at once (sum of spans / kernel span).
Build first (CPU): python tools/exp/bwd_strip_stamp.py build"""
import ctypes, os, subprocess, sys, time
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
ABL = int(os.environ.get("WABL", 0))   # FA_WIN_ABL of the stamped build (timing-only ablations, wrong grads)
SO = os.path.join(HERE, f"libbwd_stamp{ABL or ''}.so")
if len(sys.argv) > 1 and sys.argv[1] == "build":
    B = os.path.join(ROOT, "flashattention.jl_amd", "csrc", "build")
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-shared",
                    "-fno-gpu-rdc", f"-DFA_WIN_ABL={ABL}", "-o", SO, "-x", "hip", os.path.join(HERE, "bwd_strip_stamp.hip"),
                    "-x", "none", os.path.join(B, "fa_fwd.hip.o"), os.path.join(B, "fa_fwd_p4.hip.o"), os.path.join(B, "fa_bwd.hip.o"),
                    os.path.join(B, "fa_f64.hip.o")], check=True)
    sys.exit(0)
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import numpy as np, torch, fa_hip
L = ctypes.CDLL(SO)
Bimg = int(os.environ.get("WB", 32))
g = torch.Generator(device="cuda").manual_seed(1)
q, k, v, dy = (fa_hip.jl_tensor(torch.randn((128, 128, 64, Bimg), generator=g, device="cuda"), torch.bfloat16)
               for _ in range(4))
y, l, m = fa_hip.windowed_fa(q, k, v, 7)
dq, dk, dv = (torch.empty_like(q) for _ in range(3))
nwg = 3 * 19 * Bimg
out = np.zeros(24 * nwg, dtype=np.uint64)
P = lambda t: ctypes.c_void_p(t.data_ptr())
L.bwd_stamp_run.argtypes = [ctypes.c_void_p] * 10 + [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
args = (P(q), P(k), P(v), P(y), P(dy), P(l), P(m), P(dq), P(dk), P(dv), Bimg, 10)
for rep in range(3):
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 1.0:       # warm the clock on the kernel itself
        for _ in range(10):
            assert L.bwd_stamp_run(*args, None, 0) == 0
        torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        L.bwd_stamp_run(*args, None, 0)
    e1.record(); torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 10 * 1e3
    rc = L.bwd_stamp_run(*args, out.ctypes.data_as(ctypes.c_void_p), nwg)
    assert rc == 0, rc
    s = out.reshape(-1, 24).astype(np.int64)[:nwg]
    st = s[:, :16]                                 # start, loads 0..7 landed, dV 0/1, dK 0/1, dQ 0/1 stored, end
    ph = np.diff(st, axis=1)
    rt0, rt1 = s[:, 16], s[:, 17]
    clk = (s[:, 15] - s[:, 0]) / np.maximum(rt1 - rt0, 1) * 100.0
    names = [f"->L{j}" for j in range(8)] + ["->dV0", "->dV1", "->dK0", "->dK1", "->dQ0", "->dQ1", "->end"]
    print(f"abl {ABL} rep {rep}: {us:.1f} us/call; cycles between stamps (median / p90):")
    print("   " + ", ".join(f"{n}: {np.median(ph[:, i]):.0f}/{np.percentile(ph[:, i], 90):.0f}" for i, n in enumerate(names)))
    sub = np.stack([s[:, 8], s[:, 18], s[:, 19], s[:, 20], s[:, 21], s[:, 9]], axis=1)
    sd = np.diff(sub, axis=1)
    print("   within L7->dV0: " + ", ".join(f"{n}: {np.median(sd[:, i]):.0f}/{np.percentile(sd[:, i], 90):.0f}" for i, n in
          enumerate(["D, dS", "Pᵀ transpose", "dO reads", "dV MFMA + refill", "dV image + stores"])))
    print(f"   WG total cycles median {np.median(s[:, 15] - s[:, 0]):.0f}, clock {np.median(clk):.0f} MHz; WG span median "
          f"{np.median(rt1 - rt0) / 100:.2f} us", flush=True)
    span = rt1.max() - rt0.min()
    print(f"   kernel span {span / 100:.1f} us; strips in flight (sum of spans / span) {(rt1 - rt0).sum() / span:.0f}",
          flush=True)
    per = (nwg + 255) // 256                       # the launcher's persistent plan (256 CUs): consecutive strips
    G = (nwg + per - 1) // per
    sl = [slice(i * per, min((i + 1) * per, nwg)) for i in range(G)]
    wg0 = np.array([rt0[x].min() for x in sl]); wg1 = np.array([rt1[x].max() for x in sl])
    busy = np.array([(rt1[x] - rt0[x]).sum() for x in sl])
    t0m = rt0.min()
    print(f"   {G} WGs: start (us after first) median {np.median(wg0 - t0m) / 100:.1f} max {(wg0 - t0m).max() / 100:.1f}; "
          f"end median {np.median(wg1 - t0m) / 100:.1f} p10 {np.percentile(wg1 - t0m, 10) / 100:.1f} max {(wg1 - t0m).max() / 100:.1f}; "
          f"busy/lifetime median {np.median(busy / (wg1 - wg0)):.3f}", flush=True)
