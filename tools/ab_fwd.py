"""A/B the forward kernel variants in ONE process (interleaved rounds, after a
clock settle) on configs[1] and configs[3]-fwd; checks each variant against the
oracle on the first 256 rows of one slab.
Usage: python tools/ab_fwd.py [--shapes N,d,BH ...] [variants...]"""
import ctypes, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import numpy as np, torch
import fa_hip
from oracle import fa_oracle as O

L = fa_hip.lib()
L.fa_debug_set_fwd_variant.restype = ctypes.c_int
args = sys.argv[1:]
shapes = [(4096, 64, 64), (8192, 128, 64)]
if args and args[0] == "--shapes":
    shapes = []
    args = args[1:]
    while args and "," in args[0]:
        shapes.append(tuple(int(x) for x in args.pop(0).split(",")))
variants = [int(v) for v in args] or [0, 10]
PEAK = 2516.58


def mk(N, d, BH, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    out = []
    for _ in range(3):
        t = fa_hip.jl_empty((N, d, BH), torch.bfloat16)
        t.normal_(generator=g)
        out.append(t)
    return out


for (N, d, BH) in shapes:
    Q, K, V = mk(N, d, BH, 1)
    O_ = fa_hip.jl_empty((N, d, BH), torch.bfloat16)
    l = fa_hip.jl_empty((N, 1, BH)); m = fa_hip.jl_empty((N, 1, BH))
    flops = 4.0 * BH * N * N * d
    np_ = lambda t: t.float().cpu().double().numpy()
    R = min(256, N)
    ref = O.dense_fa3(np_(Q[:R, :, :1]), np_(K[:, :, :1]), np_(V[:, :, :1]))
    outs = {}
    for v in variants:
        L.fa_debug_set_fwd_variant(v)
        fa_hip.dense_fa_(O_, l, m, Q, K, V)
        torch.cuda.synchronize()
        outs[v] = (O_.clone(), l.clone(), m.clone())
        err = np.abs(np_(O_[:R, :, :1]) - ref[0]).max()
        lerr = np.abs(np_(l[:R, :, :1]) - ref[1]).max() / ref[1].max()
        merr = np.abs(np_(m[:R, :, :1]) - ref[2]).max()
        same = all(torch.equal(a, b) for a, b in zip(outs[v], outs[variants[0]]))
        dmax = (outs[v][0].float() - outs[variants[0]][0].float()).abs().max().item()
        print(f"N={N} d={d} BH={BH} variant {v}: max|dO|={err:.3e} rel|dl|={lerr:.2e} |dm|={merr:.2e}"
              f"  vs v{variants[0]}: equal={same} max|diff|={dmax:.2e}", flush=True)
    # settle: ~0.3 s of back-to-back launches before timing
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:
        for _ in range(4):
            fa_hip.dense_fa_(O_, l, m, Q, K, V)
        torch.cuda.synchronize()
    times = {v: [] for v in variants}
    for rnd in range(8):
        for v in variants:
            L.fa_debug_set_fwd_variant(v)
            for _ in range(3):
                fa_hip.dense_fa_(O_, l, m, Q, K, V)
            e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                fa_hip.dense_fa_(O_, l, m, Q, K, V)
            e1.record(); torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1) / 20 / 1e3)
    for v in variants:
        t = np.median(times[v])
        print(f"N={N} d={d} BH={BH} variant {v}: {t*1e6:.1f} us  {flops/t/1e12:.1f} TFLOP/s  "
              f"({flops/t/1e12/PEAK*100:.1f}% peak)  best {flops/min(times[v])/1e12:.1f}", flush=True)
    L.fa_debug_set_fwd_variant(0)
