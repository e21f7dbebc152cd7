"""Solo backward on larger grids: the single pass's hand-off must complete (status 0)
with no residency-check trips when the GPU is not shared.  Prints ms and status per shape.
Usage: python tools/exp/bwd_trip_check.py"""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import torch, fa_hip
for (N, d, BH) in [(16384, 128, 64), (8192, 64, 128), (4096, 64, 256), (8192, 128, 128)]:
    g = torch.Generator(device="cuda").manual_seed(3)
    mk = lambda: fa_hip.jl_tensor(torch.randn((N, d, BH), generator=g, device="cuda"), torch.bfloat16)
    Q, K, V, dO = mk(), mk(), mk(), mk()
    O, l, m = fa_hip.dense_fa(Q, K, V)
    st = []
    for rep in range(4):
        torch.cuda.synchronize(); t0 = time.perf_counter()
        fa_hip.dense_fa_backward(Q, K, V, O, dO, l, m)
        st.append(fa_hip.backward_handoff_status())
        dt = time.perf_counter() - t0
    print(f"N={N} d={d} BH={BH}: last call {dt * 1e3:.2f} ms, statuses {st}", flush=True)
    del Q, K, V, dO, O, l, m
    torch.cuda.empty_cache()
