"""configs[2]-shaped windowed BACKWARD (128x128, ws 7, d 64, bf16), B sweep, kernel paths
forced in turn by fa_debug_set_win_composed (0 auto, 3 one window per workgroup,
13 two windows per workgroup, 10 strip), in ONE process: device time per call by
HIP-graph replay, rounds interleaved, median; gradients compared bitwise to the first mode.
Usage: python tools/ab_win_bwd_modes.py [B ...]  (env WMODES="0,3,13", WROUNDS=7)"""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import torch
import fa_hip
from bench import time_graph
L = fa_hip.lib()
L.fa_debug_set_win_composed.argtypes = [ctypes.c_int]
MODES = [int(x) for x in os.environ.get("WMODES", "0,3,13").split(",")]
ROUNDS = int(os.environ.get("WROUNDS", 7))
for B in [int(x) for x in sys.argv[1:]] or [1, 2, 4]:
    g = torch.Generator(device="cuda").manual_seed(1)
    q, k, v, dy = (fa_hip.jl_tensor(torch.randn((128, 128, 64, B), generator=g, device="cuda"), torch.bfloat16)
                   for _ in range(4))
    y, l, m = fa_hip.windowed_fa(q, k, v, 7)
    bb = B * (7 * 128 * 128 * 64 * 2 + 2 * 49 * 361 * 4)
    grads, ts = {}, {c: [] for c in MODES}
    for c in MODES:
        L.fa_debug_set_win_composed(c)
        grads[c] = [t.clone() for t in fa_hip.windowed_fa_backward(q, k, v, y, dy, l, m, 7)]
        torch.cuda.synchronize()
    for _ in range(ROUNDS):
        for c in MODES:
            L.fa_debug_set_win_composed(c)
            ts[c].append(time_graph(lambda: fa_hip.windowed_fa_backward(q, k, v, y, dy, l, m, 7), 10))
    L.fa_debug_set_win_composed(0)
    for c in MODES:
        t = sorted(ts[c])[len(ts[c]) // 2]
        same = all(torch.equal(a, b) for a, b in zip(grads[c], grads[MODES[0]]))
        print(f"B={B:4d} mode {c:2d}: {t*1e6:8.2f} us  {bb/t/1e9:7.1f} GB/s  (min {min(ts[c])*1e6:.2f})  "
              f"bitwise vs mode {MODES[0]}: {same}", flush=True)
