"""After one solo single-pass backward, read the hand-off words of the workspace
(FusedFlags in fa_bwd.hip): how many wrapped slices needed bwd_dq_fast's combine
(fin == 2), the comb word, trips, and the members' XCD words.  Debugging aid."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import torch, fa_hip
al = lambda x: (x + 255) & ~255
for (N, d, BH) in [(8192, 128, 64), (4096, 64, 64)]:
    g = torch.Generator(device="cuda").manual_seed(1)
    mk = lambda: fa_hip.jl_tensor(torch.randn((N, d, BH), generator=g, device="cuda"), torch.bfloat16)
    Q, K, V, dO = mk(), mk(), mk(), mk()
    O, l, m = fa_hip.dense_fa(Q, K, V)
    for rep in range(3):
        fa_hip.dense_fa_backward(Q, K, V, O, dO, l, m)
        torch.cuda.synchronize()
        st = fa_hip.backward_handoff_status()
        dev = torch.device("cuda", torch.cuda.current_device())
        buf = fa_hip._WS[(dev.type, dev.index, torch.cuda.current_stream().cuda_stream)]
        base = al(buf.data_ptr()) - buf.data_ptr()
        w = base + 256 + al(2 * N * BH * 4)
        NS, KM = N // 64, N // 256
        words = (3 * BH * NS + BH + 2 * BH * KM + 2)
        f = buf[w:w + 4 * words].view(torch.int32).cpu()
        fin = f[2 * BH * NS:3 * BH * NS]
        serr = f[3 * BH * NS:3 * BH * NS + BH]
        xcc = f[3 * BH * NS + BH:3 * BH * NS + BH + BH * KM].reshape(BH, KM)
        prog = f[3 * BH * NS + BH + BH * KM:3 * BH * NS + BH + 2 * BH * KM].reshape(BH, KM)
        garr, comb = int(f[-2]), int(f[-1])
        print(f"N={N} d={d}: status {st}; fin==1 {int((fin == 1).sum())}, fin==2 {int((fin == 2).sum())}, "
              f"comb {comb}, trips {int(serr.sum())}, garr {garr}; slabs on one XCD "
              f"{int(((xcc == xcc[:, :1]).all(dim=1)).sum())}/{BH}; publishes per member {prog[0, :4].tolist()}", flush=True)
