"""Time diagnostic builds of the p4 forward (tools/exp/p4_abl.sh builds
libp4_lab_<tag>.so: FA_P4_ABL timing-only ablations — 1 no K/V/Q DMA in the tile loop,
2 no exponentials, 4 no LDS operand reads, 8 no softmax/max VALU; WRONG results by
design — or other -D settings) against the default kernel (variant 0) in one process,
interleaved rounds after a clock settle.
Usage: python tools/exp/p4_abl.py N,d,BH tag...   (e.g. 4096,64,64 a0 a1 pf2)"""
import ctypes, os, sys, time
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import numpy as np, torch
import fa_hip

N, d, BH = (int(x) for x in sys.argv[1].split(","))
abls = sys.argv[2:] or ["a0"]
L = fa_hip.lib()
libs = {a: ctypes.CDLL(os.path.join(HERE, f"libp4_lab_{a}.so")) for a in abls}
P = lambda t: ctypes.c_void_p(t.data_ptr())
g = torch.Generator(device="cuda").manual_seed(0)
Q, K, V = (fa_hip.jl_tensor(torch.randn((N, d, BH), generator=g, device="cuda"), torch.bfloat16) for _ in range(3))
O = torch.empty_like(Q)
l = fa_hip.jl_empty((N, 1, BH)); m = fa_hip.jl_empty((N, 1, BH))
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
flops = 4.0 * BH * N * N * d
fns = {"v0": lambda: fa_hip.dense_fa_(O, l, m, Q, K, V)}
for a, lib in libs.items():
    fns[a] = (lambda lib: lambda: lib.p4_launch(1, P(Q), P(K), P(V), P(O), P(l), P(m), N, d, BH, st))(lib)
t0 = time.perf_counter()
while time.perf_counter() - t0 < 1.0:
    for f in fns.values():
        f()
    torch.cuda.synchronize()
times = {k: [] for k in fns}
for rnd in range(6):
    for k, f in fns.items():
        f(); f()
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            f()
        e1.record(); torch.cuda.synchronize()
        times[k].append(e0.elapsed_time(e1) / 10 * 1e3)
ref = None
same = {}
for k, f in fns.items():   # bitwise check of each build's O against the default kernel's
    f(); torch.cuda.synchronize()
    if ref is None:
        ref = O.clone()
    same[k] = bool(torch.equal(O.view(torch.int16), ref.view(torch.int16)))
for k, ts in times.items():
    us = float(np.median(ts))
    print(f"N={N} d={d} BH={BH} {k}: {us:.1f} us  {flops / us / 1e6:.0f} TFLOP/s  O bitwise equal to v0: {same[k]}",
          flush=True)
