"""runcompare.py — the reference's headline benchmark table on the device.

Re-runs the reference's `runcompare(N_range=2 .^ (8:15), d_range=(64,),
bs_range=(1,), windowsize=64)` (bench/compare.jl:86-103; its published output is
logs/compare1.txt) through this library, in Float64 as the reference ran it
(bench/compare.jl:5,32,59 default T = Float64) and in bf16:

  dense_dpa / dense_fa            (N, 64, 1)
  block_dpa / block_fa            windowsize 64, stride 64, pad 0
  wind_dpa  / wind_fa             windowsize 64, stride 16, pad 0
  circ_dpa  / circ_fa             W = windowsize + 1 = 65

Every row also repeats the reference's own check (`@test O1 ≈ O2`,
bench/compare.jl:20,47,74): the device's materialising *_dpa against its *_fa,
Julia's `≈` at the element type (Float64 rows).  The reference's published
seconds (Julia Float64 on the CPU, unstated machine) are copied below as data
from logs/compare1.txt:3-9 and printed beside ours.

Also runcirculant (logs/circ_t16.txt) in Float64 and run_col_softmax
(logs/sm_cuda.txt, the reference's CUDA fused softmax) in Float32.

    python tools/runcompare.py [--dtype f64|bf16|both] > gpurun_out/runcompare.log
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flashattention.jl_amd")]

import torch  # noqa: E402

import bench  # noqa: E402  (timing plumbing: time_graph / time_region)
import fa_hip  # noqa: E402

# logs/compare1.txt:3-9 (seconds): N -> (dense_dpa, dense_fa, block_dpa, block_fa,
# wind_dpa, wind_fa, circ_dpa, circ_fa)
REFERENCE = {
    256: (0.001067, 0.000671, 0.001481, 0.001544, 0.002554, 0.001963, 0.008756, 0.010810),
    512: (0.004504, 0.002392, 0.002205, 0.001754, 0.006215, 0.005196, 0.015892, 0.009673),
    1024: (0.015696, 0.003877, 0.004517, 0.003821, 0.016184, 0.014640, 0.028846, 0.009222),
    2048: (0.056551, 0.011694, 0.008054, 0.006854, 0.029067, 0.027008, 0.059164, 0.016356),
    4096: (0.214402, 0.028642, 0.020251, 0.018076, 0.064475, 0.057028, 0.115818, 0.029273),
    8192: (0.844029, 0.092271, 0.036167, 0.033633, 0.148966, 0.136042, 0.232847, 0.055418),
    16384: (3.367637, 0.348872, 0.091136, 0.084757, 0.269094, 0.244971, 0.463745, 0.101374),
}
# logs/circ_t16.txt:3-9 (runcirculant, N 4096, d 32, bs 1, Float64, 16 threads):
# W -> (circ_dpa, circ_fa) seconds
REFERENCE_CIRC = {16: (0.021980, 0.004450), 32: (0.044041, 0.007519), 64: (0.087498, 0.015007),
                  128: (0.175385, 0.027255), 256: (0.362050, 0.058335), 512: (0.741904, 0.133951),
                  1024: (1.549231, 0.282095)}
# logs/sm_cuda.txt:2-14 (run_col_softmax, bench/softmax.jl:36-57: Float32 (M, N), dims 1,
# on the reference's CUDA GPU): (M, N) -> (naive, fused, nnlib) seconds
REFERENCE_SM = {(256, 65536): (0.001491, 0.001329, 0.000225), (512, 65536): (0.003097, 0.001456, 0.000405),
                (1024, 65536): (0.004624, 0.001843, 0.000789), (2048, 65536): (0.007390, 0.002893, 0.002418),
                (4096, 65536): (0.013122, 0.004958, 0.006674), (8192, 65536): (0.026448, 0.008687, 0.013952),
                (256, 131072): (0.011195, 0.002552, 0.000411), (512, 131072): (0.023322, 0.002800, 0.000754),
                (1024, 131072): (0.044907, 0.003602, 0.001662), (2048, 131072): (0.090770, 0.005609, 0.004767),
                (4096, 131072): (0.176741, 0.009624, 0.013177), (8192, 131072): (0.377765, 0.016920, 0.027901)}
COLS = ("dense_dpa", "dense_fa", "block_dpa", "block_fa", "wind_dpa", "wind_fa", "circ_dpa", "circ_fa")
WS = 64


def timed(fn, steps):
    try:
        return bench.time_graph(fn, steps)
    except Exception:   # not capturable: plain event-timed launches
        torch.cuda.synchronize()
        _, e = bench.time_region(fn, steps, 2)
        return e / steps


def approx(x, y, dt):
    """Julia `≈` at the element type: norm(x - y) <= sqrt(eps(T)) * max(norm(x), norm(y))."""
    x = torch.nan_to_num(x.double(), 0.0)
    y = torch.nan_to_num(y.double(), 0.0)
    eps = torch.finfo(dt).eps
    return float(torch.linalg.norm(x - y)) <= math.sqrt(eps) * max(float(torch.linalg.norm(x)),
                                                                    float(torch.linalg.norm(y)))


def run(dt, steps):
    gen = torch.Generator(device="cuda").manual_seed(0)
    rows = []
    for N in sorted(REFERENCE):
        Q, K, V = (bench._randn_jl(fa_hip, (N, 64, 1), dt, gen) for _ in range(3))
        t, ok = {}, {}
        t["dense_dpa"] = timed(lambda: fa_hip.dense_dpa(Q, K, V), steps)
        t["dense_fa"] = timed(lambda: fa_hip.dense_fa(Q, K, V), steps)
        ok["dense"] = approx(fa_hip.dense_dpa(Q, K, V)[0], fa_hip.dense_fa(Q, K, V)[0], dt)
        t["block_dpa"] = timed(lambda: fa_hip.windowed_dpa(Q, K, V, WS, WS, 0), steps)
        t["block_fa"] = timed(lambda: fa_hip.windowed_fa(Q, K, V, WS, stride=WS, pad=0), steps)
        ok["block"] = approx(fa_hip.windowed_dpa(Q, K, V, WS, WS, 0)[0],
                             fa_hip.windowed_fa(Q, K, V, WS, stride=WS, pad=0)[0], dt)
        t["wind_dpa"] = timed(lambda: fa_hip.windowed_dpa(Q, K, V, WS, 16, 0), steps)
        t["wind_fa"] = timed(lambda: fa_hip.windowed_fa(Q, K, V, WS, stride=16, pad=0), steps)
        ok["wind"] = approx(fa_hip.windowed_dpa(Q, K, V, WS, 16, 0)[0],
                            fa_hip.windowed_fa(Q, K, V, WS, stride=16, pad=0)[0], dt)
        t["circ_dpa"] = timed(lambda: fa_hip.circulant_dpa(Q, K, V, WS + 1), steps)
        t["circ_fa"] = timed(lambda: fa_hip.circulant_fa(Q, K, V, WS + 1), steps)
        ok["circ"] = approx(fa_hip.circulant_dpa(Q, K, V, WS + 1)[0], fa_hip.circulant_fa(Q, K, V, WS + 1)[0], dt)
        torch.cuda.synchronize()
        ref = dict(zip(COLS, REFERENCE[N]))
        rows.append({"N": N, "d": 64, "bs": 1, "dtype": str(dt).replace("torch.", ""),
                     "seconds": t, "dpa_approx_fa": ok,
                     "speedup_vs_reference": {c: ref[c] / t[c] for c in t}})
        print(f"{N:6d} " + " ".join(f"{t[c] * 1e3:9.4f}" for c in COLS if c in t)
              + "   ms (ref fa: " + " ".join(f"{ref[c] * 1e3:8.3f}" for c in ("dense_fa", "block_fa", "wind_fa", "circ_fa"))
              + f")  ≈ {all(ok.values())}", flush=True)
    return rows


def run_circulant(steps):
    """runcirculant (bench/compare.jl:118-130) in Float64, timed beside
    logs/circ_t16.txt (its parity is tests/test_gpu_float64.py::test_circulant_*)."""
    gen = torch.Generator(device="cuda").manual_seed(1)
    Q, K, V = (bench._randn_jl(fa_hip, (4096, 32, 1), torch.float64, gen) for _ in range(3))
    rows = []
    for W, (rdpa, rfa) in sorted(REFERENCE_CIRC.items()):
        t = timed(lambda: fa_hip.circulant_fa(Q, K, V, W), steps)
        rows.append({"W": W, "circ_fa_s": t, "reference_circ_fa_s": rfa, "speedup": rfa / t})
        print(f"circ W={W:5d}: {t * 1e3:8.4f} ms (ref {rfa * 1e3:8.3f} ms)", flush=True)
    return rows


def run_softmax(steps):
    """run_col_softmax (bench/softmax.jl:36-78): Float32 column softmax of (M, N),
    with the reference's own check fused ≈ NNlib.softmax (torch.softmax here)."""
    gen = torch.Generator(device="cuda").manual_seed(2)
    rows = []
    for (M, N), (rn, rf, rl) in sorted(REFERENCE_SM.items(), key=lambda kv: (kv[0][1], kv[0][0])):
        S = fa_hip.jl_empty((M, N, 1), torch.float32)
        S.uniform_(generator=gen)
        P = torch.empty_like(S)
        t = timed(lambda: fa_hip.fused_softmax_(P, S, 1), steps)
        fa_hip.fused_softmax_(P, S, 1)
        ref = torch.softmax(S.permute(2, 1, 0), dim=-1).permute(2, 1, 0)   # over M (dims = 1)
        ok = approx(P, ref, torch.float32)
        rows.append({"M": M, "N": N, "fused_s": t, "reference_fused_s": rf, "reference_nnlib_s": rl,
                     "speedup_vs_fused": rf / t, "approx_nnlib": ok})
        print(f"softmax M={M:5d} N={N:6d}: {t * 1e3:8.4f} ms (ref CUDA fused {rf * 1e3:7.3f}, NNlib {rl * 1e3:7.3f}) ≈ {ok}",
              flush=True)
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="both", choices=["f64", "bf16", "both"])
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    dts = {"f64": [torch.float64], "bf16": [torch.bfloat16], "both": [torch.float64, torch.bfloat16]}[a.dtype]
    out = {}
    for dt in dts:
        print(f"# {dt}: N d=64 bs=1 | " + " ".join(f"{c:>9s}" for c in COLS), flush=True)
        out[str(dt)] = run(dt, a.steps)
    circ = run_circulant(a.steps)
    sm = run_softmax(a.steps)
    print(json.dumps({"runcompare": out, "reference": "logs/compare1.txt:3-9 (Julia Float64, CPU)",
                      "runcirculant_f64": circ, "run_col_softmax_f32": sm}))


if __name__ == "__main__":
    main()
