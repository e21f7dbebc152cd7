"""(Needs the ablation hooks of tools/exp/fwd_persistent_experiment.patch.) Forward fixed (per-workgroup) cost: time configs[1]-shaped launches at several Nk with the
Q loads and/or O stores ablated (fa_debug_set_fwd_ablate; timing only, wrong results)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import numpy as np, torch
import fa_hip
L = fa_hip.lib()
N, d, BH = 4096, int(sys.argv[1]) if len(sys.argv) > 1 else 64, 64
g = torch.Generator(device="cuda").manual_seed(1)
Q = fa_hip.jl_empty((N, d, BH), torch.bfloat16); Q.copy_(torch.randn((N, d, BH), generator=g, device="cuda"))
O = fa_hip.jl_empty((N, d, BH), torch.bfloat16); l = fa_hip.jl_empty((N, 1, BH)); m = fa_hip.jl_empty((N, 1, BH))
for Nk in (64, 512, 4096):
    K = fa_hip.jl_empty((Nk, d, BH), torch.bfloat16); K.copy_(torch.randn((Nk, d, BH), generator=g, device="cuda"))
    V = fa_hip.jl_empty((Nk, d, BH), torch.bfloat16); V.copy_(torch.randn((Nk, d, BH), generator=g, device="cuda"))
    for _ in range(200): fa_hip.dense_fa_(O, l, m, Q, K, V)
    times = {a: [] for a in (0, 1, 2, 3)}
    for rnd in range(6):
        for a in times:
            L.fa_debug_set_fwd_ablate(a)
            for _ in range(3): fa_hip.dense_fa_(O, l, m, Q, K, V)
            e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20): fa_hip.dense_fa_(O, l, m, Q, K, V)
            e1.record(); torch.cuda.synchronize(); times[a].append(e0.elapsed_time(e1) / 20 * 1e3)
    L.fa_debug_set_fwd_ablate(0)
    print(f"d={d} Nk={Nk:5d}: " + "  ".join(f"abl{a} {np.median(t):7.1f} us" for a, t in times.items()), flush=True)
