"""Generate the committed golden vectors under tests/golden/*.npz.

Run from the repo root:  python tests/golden/make_golden.py

Inputs are seeded and rounded to bf16-representable values (so ONE fixture
serves the fp32, bf16 and fp16 device paths; bf16 values with |x| < 2^15 are
exact in fp16 too except for tiny subnormal cases, which randn never hits at
these scales).  Expected outputs come from oracle/fa_oracle.py (numpy
float64 restatement of the reference), which tests/test_oracle.py pins to
torch CPU sdpa / autograd / F.unfold / F.fold.  The reference itself (Julia)
cannot run here and ships no golden vectors.

Stored: inputs as bf16 bit patterns (uint16 arrays indexed by the Julia
shape), outputs as float32 (l, m as float64).
"""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import fa_oracle as O  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))


def bf16_round(x: np.ndarray) -> np.ndarray:
    """Round float64 → nearest-even bf16, returned as float64."""
    f = np.asarray(x, dtype=np.float32)
    u = f.view(np.uint32).astype(np.uint64)
    u = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return u.astype(np.uint32).view(np.float32).astype(np.float64)


def bf16_bits(x: np.ndarray) -> np.ndarray:
    return (np.asarray(x, dtype=np.float32).view(np.uint32) >> 16).astype(np.uint16)


def gen(rng, shape, kind="randn"):
    if kind == "rand":
        a = rng.random(shape)
    else:
        a = rng.standard_normal(shape)
    return bf16_round(a)


def save(name, **arrs):
    path = os.path.join(OUT, name + ".npz")
    out = {}
    for k, v in arrs.items():
        if k.startswith("in_"):
            out[k] = bf16_bits(v)            # indexed by Julia shape
        elif isinstance(v, np.ndarray) and v.dtype.kind == "f":
            out[k] = v.astype(np.float64 if k in ("l", "m") else np.float32)
        else:
            out[k] = np.asarray(v)
    np.savez_compressed(path, **out)
    return path


DENSE = [
    # name, spatial q, spatial k, d, dv, B, kind, seed
    ("dense_testjl", (30,), (30,), 12, 6, 2, "rand", 11),      # test/test.jl:6-12 shape
    ("dense_n64_d64", (64,), (64,), 64, 64, 2, "randn", 12),
    ("dense_n500_d64", (500,), (500,), 64, 64, 2, "randn", 13),
    ("dense_cfg1_n512_d64_b4", (512,), (512,), 64, 64, 4, "randn", 0),  # BASELINE configs[0] shape
    ("dense_n600_d128", (600,), (600,), 128, 128, 1, "randn", 14),
    ("dense_ragged_nq77_nk130_d64_dv32", (77,), (130,), 64, 32, 3, "randn", 15),
    ("dense_2d_12x10_d32", (12, 10), (12, 10), 32, 32, 2, "randn", 16),
    ("dense_n1000_d96_dv48", (1000,), (1000,), 96, 48, 1, "randn", 17),
]

BACKWARD = [
    ("bwd_n64_d64", 64, 64, 64, 64, 2, 21),
    ("bwd_n100_nk77_d32_dv48", 100, 77, 32, 48, 2, 22),
    ("bwd_n256_d128", 256, 256, 128, 128, 1, 23),
    ("bwd_testjl", 30, 30, 12, 6, 2, 24),
]

WINDOWED = [
    # name, spatial, d, dv, B, ws, stride, pad, seed
    ("wind_1d_n64_ws7", (64,), 16, 16, 2, 7, None, None, 31),
    ("wind_1d_n50_ws3_s2_p1", (50,), 8, 8, 2, 3, 2, 1, 32),
    ("wind_2d_20x18_ws7_cfg3like", (20, 18), 32, 32, 2, 7, 7, 3, 33),
    ("wind_2d_13x11_ws3_s2", (13, 11), 16, 8, 1, 3, 2, None, 34),
    ("block_2d_16x16_ws4", (16, 16), 16, 16, 2, 4, 4, 0, 35),
    ("wind_1d_n64_ws64_nan", (64,), 8, 8, 1, 64, None, None, 36),   # Appendix A.7: NaN tail
    ("wind_3d_6x5x4_ws3_s2", (6, 5, 4), 8, 8, 1, 3, 2, 1, 37),
]

CIRCULANT = [
    # name, N, d, dv, B, W, seed           (src/circulant.jl:9-118)
    ("circ_n30_w7_d12_dv6", 30, 12, 6, 2, 7, 41),        # N % 8 != 0: generic path
    ("circ_n64_w16_d32", 64, 32, 32, 1, 16, 42),         # even W (bench/compare.jl:98 uses W+1)
    ("circ_n20_w29_d8", 20, 8, 8, 1, 29, 43),            # W > N: keys repeat
    ("circ_n40_w57_d16", 40, 16, 16, 1, 57, 44),         # W > N on the tiled path
    ("circ_n256_w129_d64", 256, 64, 64, 2, 129, 45),     # reference bench window 128 + 1
    ("circ_n200_w1_d32_dv16", 200, 32, 16, 1, 1, 46),    # W = 1: O = V
    ("circ_n136_w64_d128_dv96", 136, 128, 96, 1, 64, 47),  # partial last workgroup
]

SOFTMAX = [
    # name, shape (M, N, B), dims, seed      (src/fused_softmax.jl:1-41)
    ("softmax_cols_37x5x2", (37, 5, 2), 1, 51),
    ("softmax_rows_37x5x2", (37, 5, 2), 2, 52),
    ("softmax_rows_300x70x1", (300, 70, 1), 2, 53),       # N > 32: two-pass row kernel
    ("softmax_cols_9000x3x1", (9000, 3, 1), 1, 54),       # M > 8192: chunked column kernel
    ("softmax_vec_1000", (1000,), 1, 55),
]


def main(which=("dense", "backward", "windowed", "circulant", "softmax")):
    if "softmax" in which:
        for name, shape, dims, seed in SOFTMAX:
            rng = np.random.default_rng(seed)
            S = gen(rng, shape) * 4.0
            print(save(name, in_s=S, p=O.fused_softmax(S, dims), dims=np.int64(dims)))
    if "circulant" in which:
        for name, N, d, dv, B, W, seed in CIRCULANT:
            rng = np.random.default_rng(seed)
            Q = gen(rng, (N, d, B)); K = gen(rng, (N, d, B)); V = gen(rng, (N, dv, B))
            Oo, l, m = O.circulant_fa3(Q, K, V, W)
            O2, _ = O.circulant_dpa3(Q, K, V, W)
            assert np.allclose(Oo, O2, rtol=1e-12, atol=1e-12)
            print(save(name, in_q=Q, in_k=K, in_v=V, o=Oo, l=l, m=m, W=np.int64(W)))
    if "dense" not in which:
        return
    for name, spq, spk, d, dv, B, kind, seed in DENSE:
        rng = np.random.default_rng(seed)
        q = gen(rng, spq + (d, B), kind)
        k = gen(rng, spk + (d, B), kind)
        v = gen(rng, spk + (dv, B), kind)
        y, l, m = O.dense_fa(q, k, v)
        y2, _ = O.dense_dpa(q, k, v)
        assert np.allclose(y, y2, rtol=1e-12, atol=1e-12)
        print(save(name, in_q=q, in_k=k, in_v=v, y=y, l=l, m=m))
    if "backward" not in which:
        return
    for name, N, Nk, d, dv, B, seed in BACKWARD:
        rng = np.random.default_rng(seed)
        Q = gen(rng, (N, d, B)); K = gen(rng, (Nk, d, B)); V = gen(rng, (Nk, dv, B))
        dO = gen(rng, (N, dv, B))
        Oo, l, m = O.dense_fa3(Q, K, V)
        dQ, dK, dV = O.dense_fa_backward(Q, K, V, Oo, dO, l, m)
        print(save(name, in_q=Q, in_k=K, in_v=V, in_do=dO, o=Oo, l=l, m=m, dq=dQ, dk=dK, dv=dV))
    if "windowed" not in which:
        return
    for name, sp, d, dv, B, ws, stride, pad, seed in WINDOWED:
        rng = np.random.default_rng(seed)
        q = gen(rng, sp + (d, B)); k = gen(rng, sp + (d, B)); v = gen(rng, sp + (dv, B))
        dy = gen(rng, sp + (dv, B))
        st = ws if stride is None else stride
        pd = (ws - 1) // 2 if pad is None else pad
        y, lw, mw = O.windowed_fa(q, k, v, ws, st, pd)
        y0 = O.windowed_dpa(q, k, v, ws, st, pd)
        assert np.allclose(np.nan_to_num(y, nan=7.0), np.nan_to_num(y0, nan=7.0), atol=1e-12)
        dq, dk, dvv = O.windowed_fa_backward(q, k, v, dy, ws, st, pd)
        print(save(name, in_q=q, in_k=k, in_v=v, in_dy=dy, y=y, l=lw, m=mw, dq=dq, dk=dk, dv=dvv,
                   ws=np.int64(ws), stride=np.int64(st), pad=np.int64(pd)))


if __name__ == "__main__":
    import sys
    main(tuple(sys.argv[1:]) or ("dense", "backward", "windowed", "circulant", "softmax"))
