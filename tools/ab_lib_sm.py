"""A/B builds of libfa_hip.so on the fused softmax (4096 x 4096 x 64 bf16, dims 1 and 2)
in ONE process, interleaved.  Usage: python tools/ab_lib_sm.py LIB_A LIB_B ..."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import numpy as np, torch
import fa_hip
from bench import _randn_jl, time_launches
paths = sys.argv[1:]
libs = []
for p in paths:
    fa_hip._LIB = None
    os.environ["FA_HIP_LIB"] = os.path.abspath(p)
    libs.append(fa_hip.lib())
g = torch.Generator(device="cuda").manual_seed(3)
S = _randn_jl(fa_hip, (4096, 4096, 64), torch.bfloat16, g)
P = torch.empty_like(S)
for dims in (1, 2):
    outs = []
    for L in libs:
        fa_hip._LIB = L
        outs.append(fa_hip.fused_softmax_(P, S, dims).clone())
    for i in range(1, len(libs)):
        print(f"dims={dims}: lib{i} vs lib0 max|diff| {float((outs[i].float() - outs[0].float()).abs().max()):.3e}", flush=True)
    del outs
    times = [[] for _ in libs]
    for rnd in range(4):
        for i, L in enumerate(libs):
            fa_hip._LIB = L
            _, e = time_launches(lambda: fa_hip.fused_softmax_(P, S, dims), 5, 2)
            times[i].append(e / 5)
    for i, p in enumerate(paths):
        t = float(np.median(times[i]))
        print(f"dims={dims} {os.path.basename(p)}: {t*1e6:8.1f} us  {2*S.numel()*2/t/1e9:7.0f} GB/s", flush=True)
