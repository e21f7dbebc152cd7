"""Compare dQ of two builds per query half (q mod 64 < 32 / >= 32) and per slab."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import torch, fa_hip
N, d, BH = (int(x) for x in os.environ.get("FA_SHAPE", "4096,128,64").split(","))
libs = []
for pth in sys.argv[1:3]:
    fa_hip._LIB = None
    os.environ["FA_HIP_LIB"] = os.path.abspath(pth)
    libs.append(fa_hip.lib())
    if os.environ.get("FA_NODIRECT"):
        libs[-1].fa_debug_set_bwd_nodirect(int(os.environ["FA_NODIRECT"]))
g = torch.Generator(device="cuda").manual_seed(1)
mk = lambda: fa_hip.jl_tensor(torch.randn((N, d, BH), generator=g, device="cuda"), torch.bfloat16)
Q, K, V, dO = mk(), mk(), mk(), mk()
fa_hip._LIB = libs[0]
O, l, m = fa_hip.dense_fa(Q, K, V)
outs = []
for L in libs:
    fa_hip._LIB = L
    r = fa_hip.dense_fa_backward(Q, K, V, O, dO, l, m)
    torch.cuda.synchronize()
    outs.append(r[0].float().cpu())
    print("status", fa_hip.backward_handoff_status(Q.device), flush=True)
a, b = outs
bad = ~torch.isclose(a, b, rtol=2e-2, atol=2e-2)   # (N, d, BH)
q = torch.arange(N)
for half in (0, 1):
    sel = ((q % 64) // 32) == half
    print(f"half {half}: bad {int(bad[sel].sum())} of {int(sel.sum()) * d * BH}, nan {int(torch.isnan(b[sel]).sum())}")
badq = bad.any(dim=1)   # (N, BH)
sl = badq.nonzero()
print("bad (query, slab) pairs", sl.shape[0])
if sl.shape[0]:
    qs = sorted(set((int(x) // 64) for x in sl[:, 0]))
    print("bad slices", qs[:40], "count", len(qs))
    print("bad slabs", sorted(set(int(x) for x in sl[:, 1]))[:20])
    print("bad feature cols in first bad row", bad[int(sl[0, 0]), :, int(sl[0, 1])].nonzero().flatten()[:40].tolist())
