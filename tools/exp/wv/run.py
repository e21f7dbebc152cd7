"""A/B of windowed forward variants (tools/exp/wv/lib_<v>_<abl>.so), configs[2] geometry."""
import ctypes, os, sys, glob
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(HERE)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import numpy as np, torch, fa_hip
names = sorted(os.path.basename(p)[4:-3] for p in glob.glob(os.path.join(HERE, "lib_*.so")))
libs = {n: ctypes.CDLL(os.path.join(HERE, f"lib_{n}.so")) for n in names}
P = lambda t: ctypes.c_void_p(t.data_ptr())
N, d, BH = 4096, 64, 64
Q, K, V = (fa_hip.jl_tensor(torch.randn((N, d, BH), device="cuda"), torch.bfloat16) for _ in range(3))
O = torch.empty_like(Q)
for Bimg in [int(x) for x in os.environ.get("WBS", "32,128").split(",")]:
    g = torch.Generator(device="cuda").manual_seed(1)
    q, k, v = (fa_hip.jl_tensor(torch.randn((128, 128, 64, Bimg), generator=g, device="cuda"), torch.bfloat16) for _ in range(3))
    ys = {}
    for n in names:
        y = torch.zeros_like(q); l = torch.zeros((49 * 361 * Bimg,), device="cuda"); m = torch.zeros_like(l)
        assert libs[n].abl_run(P(q), P(k), P(v), P(y), P(l), P(m), Bimg) == 0
        torch.cuda.synchronize(); ys[n] = (y, l, m)
    ref = [n for n in names if n.endswith("_0")][0]
    for n in names:
        if n.endswith("_0"):
            print(f"B={Bimg} {n}: bitwise y/l/m vs {ref}: {[torch.equal(a, b) for a, b in zip(ys[n], ys[ref])]}", flush=True)
    for _ in range(200):
        fa_hip.dense_fa_(O, fa_hip.jl_empty((N, 1, BH)), fa_hip.jl_empty((N, 1, BH)), Q, K, V)
    ts = {n: [] for n in names}
    y = torch.empty_like(q); l = torch.empty((49 * 361 * Bimg,), device="cuda"); m = torch.empty_like(l)
    for rnd in range(7):
        for n in names:
            f = libs[n].abl_run
            f(P(q), P(k), P(v), P(y), P(l), P(m), Bimg)
            e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                f(P(q), P(k), P(v), P(y), P(l), P(m), Bimg)
            e1.record(); torch.cuda.synchronize()
            ts[n].append(e0.elapsed_time(e1) / 20 * 1e3)
    byt = Bimg * (4 * 128 * 128 * 64 * 2 + 2 * 49 * 361 * 4)
    for n in names:
        t = float(np.median(ts[n]))
        print(f"B={Bimg} {n}: {t:.1f} us  ({byt / t / 1e3:.0f} GB/s)", flush=True)
