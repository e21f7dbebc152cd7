"""Two processes on one GPU, each timing configs[3]'s backward (8192, 128, 64 bf16), with
the single pass's slabs on one XCD each (auto) or dealt over the chip
(fa_debug_set_bwd_xcd(0)), and the split passes (9: fa_debug_set_bwd_mode(1)); plus the
solo figures.  The parent never touches the GPU:
it starts workers with Popen.
Usage: python tools/exp/bwd_two_proc_xcd.py"""
import os, subprocess, sys, time

if len(sys.argv) > 1 and sys.argv[1] == "--worker":
    xcd, t0, reps = int(sys.argv[2]), float(sys.argv[3]), int(sys.argv[4])
    ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
    import torch, fa_hip
    L = fa_hip.lib()
    if xcd == 9:
        L.fa_debug_set_bwd_mode(1)   # the split passes (no hand-off)
    else:
        L.fa_debug_set_bwd_xcd(xcd)
    g = torch.Generator(device="cuda").manual_seed(os.getpid() % 1000)
    N, d, BH = 8192, 128, 64
    mk = lambda: fa_hip.jl_tensor(torch.randn((N, d, BH), generator=g, device="cuda"), torch.bfloat16)
    Q, K, V, dO = mk(), mk(), mk(), mk()
    O, l, m = fa_hip.dense_fa(Q, K, V)
    fa_hip.dense_fa_backward(Q, K, V, O, dO, l, m)
    torch.cuda.synchronize()
    while time.time() < t0:
        time.sleep(0.001)
    st = []
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fa_hip.dense_fa_backward(Q, K, V, O, dO, l, m)
    e1.record(); torch.cuda.synchronize()
    for _ in range(2):
        fa_hip.dense_fa_backward(Q, K, V, O, dO, l, m)
        st.append(fa_hip.backward_handoff_status())
    print(f"{e0.elapsed_time(e1) / reps:.3f} {st}", flush=True)
    sys.exit(0)


def run(nproc, xcd, reps=5):
    t0 = time.time() + 40.0   # every worker past its first import torch (up to ~2 min on a fresh box)
    ps = [subprocess.Popen([sys.executable, os.path.abspath(__file__), "--worker", str(xcd), str(t0), str(reps)],
                           stdout=subprocess.PIPE, text=True) for _ in range(nproc)]
    outs = [p.communicate()[0].strip() for p in ps]
    return outs


for rnd in range(1):
    for xcd in (-1, 0, 9):
        print(f"xcd {xcd}: solo per-call ms and last statuses: {run(1, xcd)}", flush=True)
        print(f"xcd {xcd}: two processes: {run(2, xcd)}", flush=True)
