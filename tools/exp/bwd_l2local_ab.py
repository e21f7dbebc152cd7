"""A/B of the single-pass backward's hand-off forms: sc1 write-through (default) vs the
L2-local form (fa_debug_set_bwd_l2local(1)), each at chain step offsets
(fa_debug_set_bwd_hoff) 3 (default), 2 and 4; configs[3] (8192,128,64) and a d=64 shape,
interleaved rounds in one process; checks every form gives bitwise-equal dQ, dK, dV and
reports the hand-off status.  Usage: python tools/exp/bwd_l2local_ab.py"""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import numpy as np, torch, fa_hip
L = fa_hip.lib()
for (N, d, BH) in [(8192, 128, 64), (8192, 64, 64)]:
    g = torch.Generator(device="cuda").manual_seed(1)
    mk = lambda: fa_hip.jl_tensor(torch.randn((N, d, BH), generator=g, device="cuda"), torch.bfloat16)
    Q, K, V, dO = mk(), mk(), mk(), mk()
    O, l, m = fa_hip.dense_fa(Q, K, V)
    fl = 2.5 * 4.0 * BH * N * N * d
    modes = [(3, 0), (3, 1), (1, 0), (1, 1), (2, 1)]
    res, ts, st = {}, {mo: [] for mo in modes}, {}

    def setm(mo):
        L.fa_debug_set_bwd_hoff(mo[0])
        L.fa_debug_set_bwd_l2local(mo[1])
    for mode in modes:
        setm(mode)
        res[mode] = [t.clone() for t in fa_hip.dense_fa_backward(Q, K, V, O, dO, l, m)]
        st[mode] = fa_hip.backward_handoff_status()
    for rnd in range(5):
        for mode in modes:
            setm(mode)
            fa_hip.dense_fa_backward(Q, K, V, O, dO, l, m)
            e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3):
                fa_hip.dense_fa_backward(Q, K, V, O, dO, l, m)
            e1.record(); torch.cuda.synchronize()
            ts[mode].append(e0.elapsed_time(e1) / 3)
    setm((3, 0))
    L.fa_debug_set_bwd_l2local(-1)
    for mode in modes:
        eq = all(torch.equal(a, b) for a, b in zip(res[mode], res[modes[0]]))
        t = float(np.median(ts[mode]))
        print(f"N={N} d={d} BH={BH} hoff={mode[0]} l2local={mode[1]}: {t:.3f} ms  {fl / t / 1e9:.1f} TF/s  "
              f"status {st[mode]}  bitwise equal to the default form: {eq}", flush=True)
    del Q, K, V, dO, O, l, m, res
    torch.cuda.empty_cache()
