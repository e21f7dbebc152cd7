"""A/B the windowed forward + backward (configs[2] geometry: 128x128 image, ws 7, d 64,
bf16) of two or more builds of libfa_hip.so in ONE process, interleaved rounds after a
clock settle; gradients checked bitwise against the first build.
Usage: python tools/exp/ab_win_libs.py LIB_A LIB_B ... [--batches 32 8 1]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import numpy as np, torch
import fa_hip
from bench import _randn_jl

args = sys.argv[1:]
paths, batches = [], [32, 8, 1]
while args:
    a = args.pop(0)
    if a == "--batches":
        batches = []
        while args and args[0].isdigit():
            batches.append(int(args.pop(0)))
    else:
        paths.append(a)
libs = []
for p in paths:
    fa_hip._LIB = None
    os.environ["FA_HIP_LIB"] = os.path.abspath(p)
    libs.append(fa_hip.lib())


def use(i):
    fa_hip._LIB = libs[i]


g = torch.Generator(device="cuda").manual_seed(1)
N, d, BH = 4096, 64, 64   # clock settle on the dense forward
Q, K, V = (_randn_jl(fa_hip, (N, d, BH), torch.bfloat16, g) for _ in range(3))
use(0)
for _ in range(300):
    fa_hip.dense_fa(Q, K, V)
torch.cuda.synchronize()
for B in batches:
    q, k, v, dy = (_randn_jl(fa_hip, (128, 128, 64, B), torch.bfloat16, g) for _ in range(4))
    y, lw, mw = fa_hip.windowed_fa(q, k, v, 7)
    ref = [t.clone() for t in fa_hip.windowed_fa_backward(q, k, v, y, dy, lw, mw, 7)]
    tf = {i: [] for i in range(len(libs))}
    tb = {i: [] for i in range(len(libs))}
    same = {}
    for i in range(len(libs)):
        use(i)
        out = fa_hip.windowed_fa_backward(q, k, v, y, dy, lw, mw, 7)
        same[i] = all(torch.equal(a, b) for a, b in zip(out, ref))
    for rnd in range(6):
        for i in range(len(libs)):
            use(i)
            for (store, fn, reps) in ((tf, lambda: fa_hip.windowed_fa(q, k, v, 7), 20),
                                      (tb, lambda: fa_hip.windowed_fa_backward(q, k, v, y, dy, lw, mw, 7), 10)):
                fn()
                e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(reps):
                    fn()
                e1.record(); torch.cuda.synchronize()
                store[i].append(e0.elapsed_time(e1) / reps * 1e3)
    for i, p in enumerate(paths):
        print(f"B={B:3d} {os.path.basename(p)}: fwd {np.median(tf[i]):7.1f} us  bwd {np.median(tb[i]):7.1f} us  "
              f"(stream-timed, incl. launch); grads bitwise equal to the first build: {same[i]}", flush=True)
