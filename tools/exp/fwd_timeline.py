"""Launch timeline of the configs[1] forward (w8q2_wide, 512 workgroups, two per CU):
per workgroup the s_memrealtime of entry, main-loop start, main-loop end and exit,
and its CU.  Prints where the launch's time goes: dispatch spread, prologue, main
loop, epilogue, the gap between the two workgroups a CU runs, and the launch span
against the event-timed launch.  Usage: python tools/exp/fwd_timeline.py build|run"""
import ctypes, os, subprocess, sys, time
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
CS = os.path.join(ROOT, "flashattention.jl_amd", "csrc")
SO = os.path.join(HERE, "libfwd_timeline.so")
if sys.argv[1] == "build":
    objs = [os.path.join(CS, "build", f + ".o") for f in ("fa_fwd_pers.hip", "fa_fwd_p4.hip", "fa_bwd.hip", "fa_windowed.hip",
                                                          "fa_circulant.hip", "fa_softmax.hip", "fa_f64.hip")]
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-shared",
                    "-fno-gpu-rdc", "-fno-slp-vectorize", "-mllvm", "-amdgpu-sched-strategy=max-ilp",
                    "-o", SO, "-x", "hip", os.path.join(HERE, "fwd_timeline.hip"), "-x", "none"] + objs, check=True)
    sys.exit(0)
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import numpy as np, torch, fa_hip
L = ctypes.CDLL(SO)
P = lambda t: ctypes.c_void_p(t.data_ptr())
g = torch.Generator(device="cuda").manual_seed(0)
N, d, BH = 4096, 64, 64
Q, K, V = (fa_hip.jl_tensor(torch.randn((N, d, BH), generator=g, device="cuda"), torch.bfloat16) for _ in range(3))
O = torch.empty_like(Q)
l = fa_hip.jl_empty((N, 1, BH)); m = fa_hip.jl_empty((N, 1, BH))
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
launch = lambda: L.fwd_tl_launch(P(Q), P(K), P(V), P(O), P(l), P(m), N, d, BH, st)
t0 = time.perf_counter()
while time.perf_counter() - t0 < 2.0:
    for _ in range(10):
        assert launch() == 0
    torch.cuda.synchronize()
nwg = N // 512 * BH
for rep in range(3):
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    for _ in range(5):
        launch()
    e0.record(); launch(); e1.record(); torch.cuda.synchronize()
    ev = e0.elapsed_time(e1) * 1e3
    buf = np.zeros(8 * nwg, dtype=np.uint64)
    assert L.fwd_tl_read(buf.ctypes.data_as(ctypes.c_void_p), nwg) == 0
    s = buf.reshape(nwg, 8)
    t = s[:, :4].astype(np.int64)
    t = (t - t[:, 0].min()) / 100.0   # us from the first entry
    hw = s[:, 4]
    cu = ((hw >> np.uint64(32)) & np.uint64(7)).astype(np.int64) * 10000 + (hw & np.uint64(0xFFFFFFFF)).astype(np.int64) % 10000
    hwid = (hw & np.uint64(0xFFFFFFFF)).astype(np.int64)
    # HW_ID: wave_id[3:0] simd_id[5:4] pipe[7:6] cu_id[11:8] sh_id[12] se_id[15:13]...
    key = ((hw >> np.uint64(32)) & np.uint64(7)).astype(np.int64) * 4096 + ((hwid >> 8) & 0xF) + 16 * ((hwid >> 12) & 1) + 32 * ((hwid >> 13) & 7)
    med = lambda a: float(np.median(a))
    pro, loop, epi = t[:, 1] - t[:, 0], t[:, 2] - t[:, 1], t[:, 3] - t[:, 2]
    order = np.argsort(t[:, 0])
    first, second = order[: nwg // 2], order[nwg // 2:]
    gaps = []
    for k in np.unique(key):
        idx = np.where(key == k)[0]
        if len(idx) == 2:
            a, b = sorted(idx, key=lambda i: t[i, 0])
            gaps.append(t[b, 0] - t[a, 3])
    print(f"rep {rep}: event {ev:.1f} us, stamped span {t[:, 3].max():.1f} us; CUs seen {len(np.unique(key))}")
    print(f"  entry spread round 1: {np.ptp(t[first, 0]):.2f} us; round 2 entries {t[second, 0].min():.1f}..{t[second, 0].max():.1f} us")
    print(f"  prologue median {med(pro):.2f} us (round 1 {med(pro[first]):.2f}, round 2 {med(pro[second]):.2f}); "
          f"loop median {med(loop):.1f} us (r1 {med(loop[first]):.1f}, r2 {med(loop[second]):.1f}); "
          f"epilogue median {med(epi):.2f} us (r1 {med(epi[first]):.2f}, r2 {med(epi[second]):.2f})")
    if gaps:
        print(f"  exit -> next entry on the same CU: median {med(gaps):.2f} us, min {min(gaps):.2f}, max {max(gaps):.2f} ({len(gaps)} CUs)")
    print(f"  round-1 exits {t[first, 3].min():.1f}..{t[first, 3].max():.1f} us; round-2 exits {t[second, 3].min():.1f}..{t[second, 3].max():.1f} us")
