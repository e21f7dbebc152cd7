"""Phase stamps of the one-wave-per-SIMD forward (fa_fwd_p4.hip) next to the product
kernels.  Build tools/exp/libp4_lab.so first:
  hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -shared -fno-gpu-rdc -fno-slp-vectorize \
        -o tools/exp/libp4_lab.so tools/exp/p4_lab.hip
Per shape: device time of variant 0 (the default), variant 30 (fa_fwd_p4) and the stamped
build, after a clock settle; then the median over waves of the cycles in each phase of
tiles 16..19 of the first block, the block prologue / loop / epilogue / seam, and the
in-kernel clock.  Stamped-build times are diagnostic only (its fences perturb overlap).
Usage: python tools/exp/p4_lab.py [N,d,BH ...]"""
import ctypes, os, sys, time
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import numpy as np, torch
import fa_hip

L = fa_hip.lib()
L.fa_debug_set_fwd_variant.restype = ctypes.c_int
LAB = ctypes.CDLL(os.path.join(HERE, "libp4_lab.so"))
P = lambda t: ctypes.c_void_p(t.data_ptr())
shapes = [tuple(int(x) for x in a.split(",")) for a in sys.argv[1:]] or [(4096, 64, 64), (8192, 128, 64)]


def settle(fn, sec=1.0):
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < sec:
        for _ in range(8):
            fn()
        torch.cuda.synchronize()


def timeit(fn, n=20):
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


g = torch.Generator(device="cuda").manual_seed(0)
for (N, d, BH) in shapes:
    Q, K, V = (fa_hip.jl_tensor(torch.randn((N, d, BH), generator=g, device="cuda"), torch.bfloat16) for _ in range(3))
    O = torch.empty_like(Q)
    l = fa_hip.jl_empty((N, 1, BH)); m = fa_hip.jl_empty((N, 1, BH))
    flops = 4.0 * BH * N * N * d
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    def var(v):
        def f():
            L.fa_debug_set_fwd_variant(v)
            fa_hip.dense_fa_(O, l, m, Q, K, V)
            L.fa_debug_set_fwd_variant(0)
        return f
    lab = lambda: LAB.p4_launch(1, P(Q), P(K), P(V), P(O), P(l), P(m), N, d, BH, st)
    res = {}
    for rnd in range(2):
        for name, fn in (("v0", var(0)), ("v30", var(30)), ("stamped", lab)):
            settle(fn, 0.8)
            res.setdefault(name, []).append(timeit(fn))
    for name, ts in res.items():
        us = min(ts)
        print(f"N={N} d={d} BH={BH} {name}: {us:.1f} us  {flops / us / 1e6:.0f} TFLOP/s", flush=True)
    lab()
    buf = np.zeros(256 * 4 * 64, dtype=np.uint64)
    assert LAB.p4_read(buf.ctypes.data_as(ctypes.c_void_p)) == 0
    s = buf.reshape(256, 4, 64).astype(np.int64)
    med = lambda a: float(np.median(a))
    for w in range(4):
        x = s[:, w]
        t = x[:, :32].reshape(256, 4, 8)
        xph = med(t[:, :, 3] - t[:, :, 2]); yph = med(t[:, :, 5] - t[:, :, 3]); wait = med(t[:, :, 6] - t[:, :, 5])
        step = med(t[:, 1:, 2] - t[:, :-1, 2])
        bp = lambda blk, pt: x[:, 40 + 8 * blk + pt]   # block points (pt 8 of block 0 shares block 1's unused pt-0 slot)
        pro = med(bp(0, 1) - bp(0, 0)); loop = med(bp(0, 7) - bp(0, 1)); epi = med(bp(0, 8) - bp(0, 7))
        seam = med(bp(1, 1) - bp(0, 8))
        clk = (x[:, 62] - x[:, 40]) / np.maximum(x[:, 61] - x[:, 60], 1) * 100.0
        nt = N // 64
        print(f"  wave {w}: tile step {step:.0f} cyc = X {xph:.0f} + Y {yph:.0f} + wait/barrier {wait:.0f}; "
              f"block: prologue {pro:.0f}, loop {loop:.0f} ({loop / max(nt - 1, 1):.0f}/tile), epilogue {epi:.0f}, "
              f"seam->next loop {seam:.0f}; clock {med(clk):.0f} MHz", flush=True)
    del Q, K, V, O, l, m
    torch.cuda.empty_cache()
