"""Per-workgroup phase cycles of the strip windowed forward (win_strip, mode 10) at
configs[2] (128x128, ws 7, d 64, bf16), B = 32 by default: s_memtime cycles per
phase (median / p90 over workgroups), the in-kernel clock, the workgroup realtime
span, and how many workgroups ran at once (sum of spans / kernel span).
Build first (CPU): python tools/exp/strip_stamp.py build"""
import ctypes, os, subprocess, sys, time
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
ABL = int(os.environ.get("WABL", 0))   # FA_WIN_ABL of the stamped build (timing-only ablations, wrong y)
SO = os.path.join(HERE, f"libstrip_stamp{ABL or ''}.so")
if len(sys.argv) > 1 and sys.argv[1] == "build":
    B = os.path.join(ROOT, "flashattention.jl_amd", "csrc", "build")
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-shared",
                    "-fno-gpu-rdc", f"-DFA_WIN_ABL={ABL}", "-o", SO, "-x", "hip", os.path.join(HERE, "strip_stamp.hip"),
                    "-x", "none", os.path.join(B, "fa_fwd.hip.o"), os.path.join(B, "fa_fwd_p4.hip.o"), os.path.join(B, "fa_bwd.hip.o"),
                    os.path.join(B, "fa_f64.hip.o")], check=True)
    sys.exit(0)
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import numpy as np, torch, fa_hip
L = ctypes.CDLL(SO)
Bimg = int(os.environ.get("WB", 32))
g = torch.Generator(device="cuda").manual_seed(1)
q, k, v = (fa_hip.jl_tensor(torch.randn((128, 128, 64, Bimg), generator=g, device="cuda"), torch.bfloat16) for _ in range(3))
y = torch.empty_like(q)
l = torch.empty((49 * 361 * Bimg,), device="cuda"); m = torch.empty_like(l)
nwg = 3 * 19 * Bimg
out = np.zeros(8 * nwg, dtype=np.uint64)
P = lambda t: ctypes.c_void_p(t.data_ptr())
wsb = 64 << 20
wst = torch.empty(wsb, dtype=torch.uint8, device="cuda")
L.strip_stamp_run.argtypes = [ctypes.c_void_p] * 6 + [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                                      ctypes.c_void_p, ctypes.c_size_t]
for rep in range(3):
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 1.0:       # warm the clock on the kernel itself
        for _ in range(20):
            assert L.strip_stamp_run(P(q), P(k), P(v), P(y), P(l), P(m), Bimg, 10, None, 0, P(wst), wsb) == 0
        torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        L.strip_stamp_run(P(q), P(k), P(v), P(y), P(l), P(m), Bimg, 10, None, 0, P(wst), wsb)
    e1.record(); torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 20 * 1e3
    rc = L.strip_stamp_run(P(q), P(k), P(v), P(y), P(l), P(m), Bimg, 10, out.ctypes.data_as(ctypes.c_void_p), nwg, P(wst), wsb)
    assert rc == 0, rc
    s = out.reshape(-1, 8).astype(np.int64)[:nwg]
    ph = np.diff(s[:, :6], axis=1)
    rt0, rt1 = s[:, 6], s[:, 7]
    clk = (s[:, 5] - s[:, 0]) / np.maximum(rt1 - rt0, 1) * 100.0
    names = ["first chunk", "QK", "softmax + V", "PV + y (chunk 0)", "PV + y (chunk 1)"]
    print(f"abl {ABL} rep {rep}: {us:.1f} us/call; per-WG phase cycles (median / p90): " +
          ", ".join(f"{n}: {np.median(ph[:, i]):.0f}/{np.percentile(ph[:, i], 90):.0f}" for i, n in enumerate(names)))
    span = rt1.max() - rt0.min()
    print(f"   WG total cycles median {np.median(s[:, 5] - s[:, 0]):.0f}, clock {np.median(clk):.0f} MHz; WG span median "
          f"{np.median(rt1 - rt0) / 100:.2f} us; kernel span {span / 100:.1f} us; WGs in flight (sum of spans / span) "
          f"{(rt1 - rt0).sum() / span:.0f}", flush=True)
