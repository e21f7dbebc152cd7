"""In-kernel cycles and clock of the dense forward (MI355X_MICROARCH
'DVFS give-back' item 6): builds tools/exp/fwd_stamp.hip once per ablation
(FA_FWD_ABL 0 = the product code; 1 no exp, 2 no row sum, 4 no row max, 7 all three;
timing-only, WRONG results), then per build and variant: >= SETTLE s of back-to-back
launches on random data, device time per launch (HIP events), and from the stamps of
one launch: cycles per 64-key tile of the main loop, prologue and epilogue cycles,
and the in-kernel clock = d(s_memtime) / d(s_memrealtime) x 100 MHz (median over
workgroups).  Usage:  python tools/exp/fwd_stamp.py build [abl ...]
                      python tools/exp/fwd_stamp.py run   [abl ...]"""
import ctypes, os, subprocess, sys, time
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
CS = os.path.join(ROOT, "flashattention.jl_amd", "csrc")
so = lambda abl: os.path.join(HERE, f"libfwd_stamp{abl}.so")
abls = [int(a) for a in sys.argv[2:]] or [0]
if sys.argv[1] == "build":
    objs = [os.path.join(CS, "build", f + ".o") for f in ("fa_bwd.hip", "fa_windowed.hip", "fa_circulant.hip",
                                                          "fa_softmax.hip", "fa_f64.hip")]
    for abl in abls:
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-shared",
                        "-fno-gpu-rdc", "-fno-slp-vectorize", "-mllvm", "-amdgpu-sched-strategy=max-ilp",
                        f"-DFA_FWD_ABL={abl}", "-o", so(abl), "-x", "hip", os.path.join(HERE, "fwd_stamp.hip"),
                        "-x", "none"] + objs, check=True)
    sys.exit(0)

sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]
import numpy as np, torch, fa_hip
SETTLE = float(os.environ.get("SETTLE", "2.0"))
variants = [int(v) for v in os.environ.get("FVARS", "0").split(",")]
shapes = [(4096, 64, 64), (8192, 128, 64)] if os.environ.get("FD128", "1") == "1" else [(4096, 64, 64)]
libs = {abl: ctypes.CDLL(so(abl)) for abl in abls}
P = lambda t: ctypes.c_void_p(t.data_ptr())
g = torch.Generator(device="cuda").manual_seed(0)
for (N, d, BH) in shapes:
    Q, K, V = (fa_hip.jl_tensor(torch.randn((N, d, BH), generator=g, device="cuda"), torch.bfloat16) for _ in range(3))
    O = torch.empty_like(Q)
    l = fa_hip.jl_empty((N, 1, BH)); m = fa_hip.jl_empty((N, 1, BH))
    flops = 4.0 * BH * N * N * d
    ntile = N // 64
    for rnd in range(2):
        for abl, L in libs.items():
            for var in variants:
                st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
                launch = lambda: L.fwd_stamp_launch(var, P(Q), P(K), P(V), P(O), P(l), P(m), N, d, BH, st)
                t0 = time.perf_counter(); n = 0
                while time.perf_counter() - t0 < SETTLE:
                    for _ in range(10):
                        assert launch() == 0
                    n += 10
                    torch.cuda.synchronize()
                e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(20):
                    launch()
                e1.record(); torch.cuda.synchronize()
                us = e0.elapsed_time(e1) / 20 * 1e3
                rows = 512 if (d <= 64 and var in (0, 7, 20)) else 256
                nwg = N // rows * BH
                buf = np.zeros(16 * nwg, dtype=np.uint64)
                assert L.fwd_stamp_read(buf.ctypes.data_as(ctypes.c_void_p), nwg) == 0
                s = buf.reshape(nwg, 2, 8).astype(np.int64)
                med = lambda a: float(np.median(a))
                out = []
                for hf, nm in ((0, "w0"), (1, "w4")):
                    x = s[:, hf]
                    pro, loop, epi = x[:, 1] - x[:, 0], x[:, 2] - x[:, 1], x[:, 3] - x[:, 2]
                    clk = (x[:, 3] - x[:, 0]) / np.maximum(x[:, 7] - x[:, 6], 1) * 100.0
                    out.append(f"{nm}: prologue {med(pro):.0f} cyc, loop {med(loop) / ntile:.0f} cyc/tile, "
                               f"epilogue {med(epi):.0f} cyc, clock {med(clk):.0f} MHz")
                span = (s[:, 0, 7].max() - s[:, 0, 6].min()) / 100.0
                print(f"N={N} d={d} abl={abl} var={var} rnd={rnd}: {us:.1f} us ({flops / us / 1e6:.0f} TFLOP/s) "
                      f"after {n} settle launches; " + "; ".join(out) + f"; kernel span {span:.1f} us", flush=True)
