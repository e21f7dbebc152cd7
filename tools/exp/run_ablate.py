"""Time the ablation variants of the v2 forward on configs[1] (one process, interleaved)."""
import ctypes, os, sys
import numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import fa_hip
L = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libfwd_ablate.so"))
L.abl_fwd_launch.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 6 + [ctypes.c_int] * 3 + [ctypes.c_void_p]
N, d, BH = 4096, 64, 64
g = torch.Generator(device="cuda").manual_seed(1)
Q, K, V = [fa_hip.jl_empty((N, d, BH), torch.bfloat16) for _ in range(3)]
for t in (Q, K, V): t.copy_(torch.randn((N, d, BH), generator=g, device="cuda"))
O = fa_hip.jl_empty((N, d, BH), torch.bfloat16); l = fa_hip.jl_empty((N, 1, BH)); m = fa_hip.jl_empty((N, 1, BH))
names = {0: "full", 1: "no exp", 2: "no tile loads", 4: "no PV mfma", 8: "no QK mfma", 16: "no softmax(exp+fma)",
         32: "no barrier(racy)", 3: "no exp+loads", 7: "no exp/loads/PV", 12: "no mfma at all", 5: "no exp+PV",
         17: "no exp, no fma", 34: "no loads, no barrier", 14: "no mfma, no loads", 28: "no mfma, no softmax",
         30: "no mfma/loads/softmax", 76: "no mfma, no K reads", 140: "no mfma, no V reads", 204: "no mfma, no LDS reads",
         206: "no mfma/LDS rd/loads", 222: "only barrier+cvt+misc", 64: "no K LDS reads", 128: "no V LDS reads",
         192: "no LDS reads", 194: "no LDS reads, no loads"}
abls = [int(a) for a in sys.argv[1:]] or list(names)
st = torch.cuda.current_stream().cuda_stream
P = lambda t: ctypes.c_void_p(t.data_ptr())
times = {a: [] for a in abls}
for rnd in range(5):
    for a in abls:
        for _ in range(2): L.abl_fwd_launch(a, P(Q), P(K), P(V), P(O), P(l), P(m), N, N, BH, ctypes.c_void_p(st))
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10): L.abl_fwd_launch(a, P(Q), P(K), P(V), P(O), P(l), P(m), N, N, BH, ctypes.c_void_p(st))
        e1.record(); torch.cuda.synchronize()
        times[a].append(e0.elapsed_time(e1) / 10)
fl = 4.0 * BH * N * N * d
for a in abls:
    t = np.median(times[a]) / 1e3
    print(f"abl {a:3d} {names.get(a, ''):24s} {t*1e6:8.1f} us  {fl/t/1e12:7.1f} TF-equiv")
