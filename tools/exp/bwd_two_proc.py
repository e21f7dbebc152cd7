"""Two processes on one GPU, each timing configs[3]'s backward (8192, 128, 64 bf16), for
residency-check windows (fa_debug_set_bwd_stall_us) given on the command line; plus
the solo figure.  The parent never touches the GPU: it starts workers with Popen.
Usage: python tools/exp/bwd_two_proc.py [stall_us ...]"""
import os, subprocess, sys, time

if len(sys.argv) > 1 and sys.argv[1] == "--worker":
    stall, t0, reps = int(sys.argv[2]), float(sys.argv[3]), int(sys.argv[4])
    ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
    import torch, fa_hip
    L = fa_hip.lib()
    L.fa_debug_set_bwd_stall_us(stall)
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


def run(nproc, stall, reps=5):
    t0 = time.time() + 40.0   # every worker past its first import torch (up to ~2 min on a fresh box)
    ps = [subprocess.Popen([sys.executable, os.path.abspath(__file__), "--worker", str(stall), str(t0), str(reps)],
                           stdout=subprocess.PIPE, text=True) for _ in range(nproc)]
    outs = [p.communicate()[0].strip() for p in ps]
    return outs


stalls = [int(x) for x in sys.argv[1:]] or [50, 200, 1000]
print("solo, stall 50 us:", run(1, 50), flush=True)
for s in stalls:
    print(f"two processes, stall {s} us: per-call ms and last statuses: {run(2, s)}", flush=True)
