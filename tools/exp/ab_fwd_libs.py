"""A/B the dense forward of two builds of libfa_hip.so in ONE process, interleaved
rounds after a clock settle: configs[1] (4096, 64, 64 slabs) bf16 and a ragged-key
shape; y, l, m checked bitwise against the first build.
Usage: python tools/exp/ab_fwd_libs.py LIB_A LIB_B"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import torch
import fa_hip
from bench import _randn_jl

libs = []
for p in sys.argv[1:]:
    fa_hip._LIB = None
    os.environ["FA_HIP_LIB"] = os.path.abspath(p)
    libs.append(fa_hip.lib())


def use(i):
    fa_hip._LIB = libs[i]


g = torch.Generator(device="cuda").manual_seed(1)
shapes = [(4096, 4096, 64, 64), (4096, 4000, 64, 64), (8192, 8192, 128, 64)]
data = {}
for (N, Nk, d, BH) in shapes:
    data[(N, Nk, d, BH)] = (_randn_jl(fa_hip, (N, d, BH), torch.bfloat16, g), _randn_jl(fa_hip, (Nk, d, BH), torch.bfloat16, g),
                            _randn_jl(fa_hip, (Nk, d, BH), torch.bfloat16, g))
use(0)
Q, K, V = data[shapes[0]]
for _ in range(2000):
    fa_hip.dense_fa(Q, K, V)
torch.cuda.synchronize()
for sh in shapes:
    Q, K, V = data[sh]
    ref = None
    same = {}
    for i in range(len(libs)):
        use(i)
        out = [t.clone() for t in fa_hip.dense_fa(Q, K, V)]
        ref = ref or out
        same[i] = all(torch.equal(a, b) for a, b in zip(out, ref))
    ts = {i: [] for i in range(len(libs))}
    for rnd in range(8):
        for i in range(len(libs)):
            use(i)
            for _ in range(20):
                fa_hip.dense_fa(Q, K, V)
            e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(40):
                fa_hip.dense_fa(Q, K, V)
            e1.record(); torch.cuda.synchronize()
            ts[i].append(e0.elapsed_time(e1) / 40 * 1e3)
    N, Nk, d, BH = sh
    fl = 4.0 * BH * N * Nk * d
    for i in range(len(libs)):
        v = sorted(ts[i])
        print(f"{sh} lib {i}: median {v[len(v) // 2]:8.1f} us  best {v[0]:8.1f}  ({fl / v[len(v) // 2] / 1e6:6.0f} TFLOP/s)  "
              f"bitwise equal to lib 0: {same[i]}", flush=True)
