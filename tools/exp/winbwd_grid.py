"""Strip windowed backward (configs[2] shape, B = 32 by default) against its grid size
(fa_debug_set_win_bwd_grid): device time by HIP-graph replay, interleaved rounds, median;
gradients bitwise against the default grid.  Usage: python tools/exp/winbwd_grid.py [grids...]"""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import torch, fa_hip
from bench import time_graph
L = fa_hip.lib()
L.fa_debug_set_win_bwd_grid.argtypes = [ctypes.c_int]
grids = [int(x) for x in sys.argv[1:]] or [0, 240, 224, 192, 128]
B = int(os.environ.get("WB", 32))
g = torch.Generator(device="cuda").manual_seed(1)
q, k, v, dy = (fa_hip.jl_tensor(torch.randn((128, 128, 64, B), generator=g, device="cuda"), torch.bfloat16) for _ in range(4))
y, l, m = fa_hip.windowed_fa(q, k, v, 7)
bb = B * (7 * 128 * 128 * 64 * 2 + 2 * 49 * 361 * 4)
ref, ts = None, {gr: [] for gr in grids}
for gr in grids:
    L.fa_debug_set_win_bwd_grid(gr)
    out = [t.clone() for t in fa_hip.windowed_fa_backward(q, k, v, y, dy, l, m, 7)]
    torch.cuda.synchronize()
    if ref is None:
        ref = out
    print(f"grid {gr}: bitwise vs first: {all(torch.equal(a, b) for a, b in zip(out, ref))}", flush=True)
for _ in range(int(os.environ.get("WROUNDS", 7))):
    for gr in grids:
        L.fa_debug_set_win_bwd_grid(gr)
        ts[gr].append(time_graph(lambda: fa_hip.windowed_fa_backward(q, k, v, y, dy, l, m, 7), 10))
L.fa_debug_set_win_bwd_grid(0)
for gr in grids:
    t = sorted(ts[gr])[len(ts[gr]) // 2]
    print(f"B={B} grid {gr:4d}: {t*1e6:8.2f} us  {bb/t/1e9:7.1f} GB/s  (min {min(ts[gr])*1e6:.2f})", flush=True)
