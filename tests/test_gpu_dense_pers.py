"""GPU parity of the persistent 8-wave forward at head dims <= 64 (csrc/fa_fwd_pers.hip,
fa_debug_set_fwd_variant(40)).  Its tile body is the 8-wave kernel's (w8q2_wide,
variant 7) in the same order — the reference's dense_fa! update, src/dense.jl:21-102,
online softmax :78-91 — so y, l and m must be BITWISE equal to that kernel's on every
slab, and within the bf16 / f16 tolerance of the float64 oracle.  The shapes exercise
what the persistent grid adds: workgroups that take one, two or more 512-row blocks
and unequal numbers of them, K/V streams and Q prefetches crossing slab boundaries,
partial last query blocks, head dims padded to their class (d = 48, dv = 32, d = 32),
the minimum of 8 key tiles per block, and the O pieces of one block leaving while the
next block's Q arrives over them."""
from __future__ import annotations

import ctypes

import numpy as np
import pytest
import torch

from conftest import assert_close, assert_lm_close
from oracle import fa_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def fa():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm device")
    import fa_hip
    fa_hip.lib()
    return fa_hip


def _np(t):
    return t.float().cpu().double().numpy()


def _run(fa, variant, Q, K, V):
    L = fa.lib()
    L.fa_debug_fwd_last_path.restype = ctypes.c_int
    old = L.fa_debug_set_fwd_variant(variant)
    try:
        y, l, m = fa.dense_fa(Q, K, V)
        torch.cuda.synchronize()
        path = L.fa_debug_fwd_last_path()
    finally:
        L.fa_debug_set_fwd_variant(old)
    return y, l, m, path


# (N, Nk, d, dv, B, dtype)
SHAPES = [
    (4096, 4096, 64, 64, 64, "bfloat16"),   # configs[1]: 512 blocks, two per workgroup
    (4096, 1024, 64, 64, 96, "bfloat16"),   # 768 blocks: three per workgroup
    (1000, 512, 64, 64, 300, "bfloat16"),   # partial last block (1000 = 512 + 488), 8 key tiles, 600 blocks
    (2048, 2048, 64, 64, 40, "float16"),    # f16, 160 blocks: fewer than the CUs, one each
    (2048, 1536, 64, 64, 77, "bfloat16"),   # 308 blocks: some workgroups take two, others one
    (1536, 1280, 48, 32, 200, "bfloat16"),  # d = 48 (class 64), dv = 32: 600 blocks
    (1024, 1024, 32, 64, 300, "float16"),   # d = 32, dv = 64, f16
]


@pytest.mark.parametrize("N,Nk,d,dv,B,dtype", SHAPES)
def test_pers_bitwise_vs_8wave_and_oracle(fa, N, Nk, d, dv, B, dtype):
    dt = torch.bfloat16 if dtype == "bfloat16" else torch.float16
    rng = np.random.default_rng(N + Nk + d + dv + B)
    cast = lambda a: torch.tensor(a).to(dt)
    q, k, v = (rng.standard_normal(sh) for sh in ((N, d, B), (Nk, d, B), (Nk, dv, B)))
    Q, K, V = (fa.jl_tensor(cast(a).double().numpy(), dt) for a in (q, k, v))
    y40, l40, m40, path40 = _run(fa, 40, Q, K, V)
    assert path40 == 40, "the shape meets the persistent kernel's launch rules, so variant 40 must run it"
    y7, l7, m7, path7 = _run(fa, 7, Q, K, V)
    assert path7 == 0
    assert torch.equal(y40.view(torch.int16), y7.view(torch.int16)), "y not bitwise equal to the 8-wave kernel"
    assert torch.equal(l40, l7) and torch.equal(m40, m7), "l, m not bitwise equal to the 8-wave kernel"
    # the oracle on three slabs: the first, one in the middle and the last (different
    # workgroups, blocks late in a workgroup's walk)
    for b in sorted({0, B // 2, B - 1}):
        qs, ks, vs = (cast(a[..., b:b + 1]).double().numpy() for a in (q, k, v))
        yr, lr, mr = O.dense_fa3(qs, ks, vs)
        assert_close(_np(y40[..., b:b + 1]), yr, dtype, f"y slab {b}")
        assert_lm_close(_np(l40[..., b:b + 1]), lr, dtype, f"l slab {b}")
        assert_lm_close(_np(m40[..., b:b + 1]), mr, dtype, f"m slab {b}")


@pytest.mark.parametrize("thr", [8.0, 0.0])
def test_pers_rescale_branch(fa, thr):
    """Running maxima that climb over the key sweep (every tile rescales at threshold 0)
    plus spike keys, on 640 blocks: bitwise equal to the 8-wave kernel at the same
    threshold, and within tolerance of the oracle."""
    L = fa.lib()
    rng = np.random.default_rng(31)
    N, Nk, d, B = 1024, 1024, 64, 320
    u = rng.standard_normal(d); u /= np.linalg.norm(u)
    q = np.repeat((u * 6.0)[None, :, None], N, 0).repeat(B, 2) + 0.3 * rng.standard_normal((N, d, B))
    t = np.linspace(-1.0, 1.0, Nk) * 24.0
    k = t[:, None, None] * u[None, :, None] + 0.3 * rng.standard_normal((Nk, d, B))
    k[700] = q[10] * 5.0
    k[1000, :, 3] = q[600, :, 3] * 7.0
    v = rng.uniform(-4, 4, (Nk, d, B))
    bf = lambda a: torch.tensor(a).to(torch.bfloat16).double().numpy()
    q, k, v = bf(q), bf(k), bf(v)
    Q, K, V = (fa.jl_tensor(a, torch.bfloat16) for a in (q, k, v))
    old = L.fa_debug_set_rescale_threshold(thr)
    try:
        y40, l40, m40, path40 = _run(fa, 40, Q, K, V)
        y7, l7, m7, _ = _run(fa, 7, Q, K, V)
    finally:
        L.fa_debug_set_rescale_threshold(old)
    assert path40 == 40
    assert torch.equal(y40.view(torch.int16), y7.view(torch.int16)), "y not bitwise equal"
    assert torch.equal(l40, l7) and torch.equal(m40, m7), "l, m not bitwise equal"
    for b in (0, 3):
        yr, lr, mr = O.dense_fa3(q[..., b:b + 1], k[..., b:b + 1], v[..., b:b + 1])
        assert_close(_np(y40[..., b:b + 1]), yr, "bfloat16", f"y slab {b}")
        assert_lm_close(_np(l40[..., b:b + 1]), lr, "bfloat16", f"l slab {b}")
        assert_lm_close(_np(m40[..., b:b + 1]), mr, "bfloat16", f"m slab {b}")


def test_pers_falls_back_outside_its_rules(fa):
    """Shapes outside the persistent kernel's rules (key count not a multiple of 128,
    fewer than 8 key tiles, d = 128) run the other kernels under variant 40, with the
    default kernels' results."""
    rng = np.random.default_rng(5)
    for (N, Nk, d, B) in ((1024, 1088, 64, 128), (1024, 384, 64, 128), (1024, 1024, 128, 64)):
        Q, K, V = (fa.jl_tensor(rng.standard_normal(sh), torch.bfloat16)
                   for sh in ((N, d, B), (Nk, d, B), (Nk, d, B)))
        y40, l40, m40, path40 = _run(fa, 40, Q, K, V)
        assert path40 != 40, (N, Nk, d, B)
        y0, l0, m0, _ = _run(fa, 0, Q, K, V)
        assert torch.equal(y40, y0) and torch.equal(l40, l0) and torch.equal(m40, m0)
