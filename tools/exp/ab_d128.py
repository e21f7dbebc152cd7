"""A/B forward variants at d=128: configs[3] (8192,128,64), configs[4]'s per-GPU share
(16384,128,128) and (4096,128,64), interleaved rounds in one process."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import numpy as np, torch, fa_hip
L = fa_hip.lib()
variants = [int(v) for v in sys.argv[1:]] or [5, 8]
for (N, d, BH) in [(8192, 128, 64), (16384, 128, 128), (4096, 128, 64)]:
    g = torch.Generator(device="cuda").manual_seed(1)
    Q, K, V = (fa_hip.jl_tensor(torch.randn((N, d, BH), generator=g, device="cuda"), torch.bfloat16) for _ in range(3))
    O = fa_hip.jl_empty((N, d, BH), torch.bfloat16); l = fa_hip.jl_empty((N, 1, BH)); m = fa_hip.jl_empty((N, 1, BH))
    fl = 4.0 * BH * N * N * d
    ts = {v: [] for v in variants}
    outs = {}
    for v in variants:
        L.fa_debug_set_fwd_variant(v); fa_hip.dense_fa_(O, l, m, Q, K, V); torch.cuda.synchronize()
        outs[v] = O[:, :, :2].float().clone()
    for rnd in range(5):
        for v in variants:
            L.fa_debug_set_fwd_variant(v)
            fa_hip.dense_fa_(O, l, m, Q, K, V)
            e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(4): fa_hip.dense_fa_(O, l, m, Q, K, V)
            e1.record(); torch.cuda.synchronize(); ts[v].append(e0.elapsed_time(e1) / 4 / 1e3)
    base = variants[0]
    for v in variants:
        t = np.median(ts[v])
        print(f"N={N} BH={BH} variant {v}: {fl/t/1e12:7.1f} TF/s  max|dO vs {base}| {float((outs[v]-outs[base]).abs().max()):.2e}", flush=True)
    L.fa_debug_set_fwd_variant(0)
