"""Cycles per 4 MFMA slots through one tile's X/Y stream of the p4 forward (slot-stamp
builds libp4_lab_<tag>.so from tools/exp/p4_abl.sh with -DP4_SLOTS): s_memtime sampled
at slots 0, 4, 8, ... of tile 16 of each workgroup's first block, median over waves.
Usage: python tools/exp/p4_slots.py N,d,BH tag..."""
import ctypes, os, sys, time
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import numpy as np, torch
import fa_hip

N, d, BH = (int(x) for x in sys.argv[1].split(","))
tags = sys.argv[2:] or ["s0"]
fa_hip.lib()
P = lambda t: ctypes.c_void_p(t.data_ptr())
g = torch.Generator(device="cuda").manual_seed(0)
Q, K, V = (fa_hip.jl_tensor(torch.randn((N, d, BH), generator=g, device="cuda"), torch.bfloat16) for _ in range(3))
O = torch.empty_like(Q)
l = fa_hip.jl_empty((N, 1, BH)); m = fa_hip.jl_empty((N, 1, BH))
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
nsamp = 2 * (2 * d // 16 + 4 * d // 32) // 4     # X/Y stream slots / 4
for tag in tags:
    L = ctypes.CDLL(os.path.join(HERE, f"libp4_lab_{tag}.so"))
    run = lambda: L.p4_launch(1, P(Q), P(K), P(V), P(O), P(l), P(m), N, d, BH, st)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 1.0:
        for _ in range(5):
            run()
        torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        run()
    e1.record(); torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 10 * 1e3
    run()
    buf = np.zeros(256 * 4 * 16, dtype=np.uint64)
    assert L.p4_read_slots(buf.ctypes.data_as(ctypes.c_void_p)) == 0
    s = buf.reshape(256 * 4, 16).astype(np.int64)[:, :nsamp]
    dl = np.diff(s, axis=1)
    med = np.median(dl, axis=0)
    p90 = np.percentile(dl, 90, axis=0)
    print(f"{tag} N={N} d={d}: {us:.1f} us; cycles per 4 slots (median/p90), X then Y: " +
          " ".join(f"{a:.0f}/{b:.0f}" for a, b in zip(med, p90)) + f"; sum {med.sum():.0f}", flush=True)
