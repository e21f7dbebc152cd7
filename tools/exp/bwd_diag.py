"""Single-pass backward vs split passes on small shapes: which of dQ, dK, dV differ, and
where (slice, feature) — a debugging aid.  Usage: python tools/exp/bwd_diag.py"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import torch, fa_hip
L = fa_hip.lib()
for (N, Nk, d, dv, B) in [(256, 256, 32, 32, 4), (256, 256, 64, 64, 4), (512, 256, 32, 32, 2), (512, 512, 32, 32, 2),
                          (256, 256, 32, 32, 1), (512, 512, 64, 64, 2)]:
    g = torch.Generator(device="cuda").manual_seed(1)
    mk = lambda n, c: fa_hip.jl_tensor(torch.randn((n, c, B), generator=g, device="cuda"), torch.bfloat16)
    Q, K, V, dO = mk(N, d), mk(Nk, d), mk(Nk, dv), mk(N, dv)
    O, l, m = fa_hip.dense_fa(Q, K, V)
    res = {}
    for mode in (2, 1):
        L.fa_debug_set_bwd_mode(mode)
        res[mode] = [t.float() for t in fa_hip.dense_fa_backward(Q, K, V, O, dO, l, m)]
        torch.cuda.synchronize()
        st = fa_hip.backward_handoff_status()
        res[mode].append(st)
    L.fa_debug_set_bwd_mode(0)
    out = []
    for i, nm in enumerate(("dQ", "dK", "dV")):
        a, b = res[2][i], res[1][i]
        err = (a - b).abs().max().item() / b.abs().max().item()
        out.append(f"{nm} {err:.2e}")
        if nm == "dQ" and err > 1e-2:
            e = (a - b).abs()   # (N, d, B)
            per_slice = e.reshape(N // 64, 64, d, B).amax(dim=(1, 2))
            out.append("dQ err per (slice, slab): " + str(per_slice.cpu().numpy().round(2).tolist()))
            per_f = e.amax(dim=(0, 2))
            out.append("dQ err per feature: " + str(per_f.cpu().numpy().round(1).tolist()))
            out.append(f"|a| max {a.abs().max().item():.3g} |b| max {b.abs().max().item():.3g}")
    print((N, Nk, d, dv, B), "status", res[2][3], res[1][3], "; ".join(out), flush=True)
