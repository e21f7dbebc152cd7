"""GPU parity of the one-wave-per-SIMD persistent forward (csrc/fa_fwd_p4.hip,
fa_debug_set_fwd_variant(30)).  It computes the reference's dense_fa! update
(src/dense.jl:21-102; online softmax :78-91) with the same arithmetic in the same
order as the 8-wave kernels (w8q2_wide at d = 64, w8b64_wide at d = 128: variants 7
and 5), so its y, l and m must be BITWISE equal to theirs, on every slab, and within
the bf16 tolerance of the float64 oracle.  Shapes follow its launch rules: whole
64-key tiles, N % 8 == 0, at least one 256-row block per CU, and enough key tiles for
the next block's Q prefetch; they cover a partial last query block, workgroups that
take unequal numbers of blocks, and K / V streams crossing slab boundaries."""
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


# (N, Nk, d, B, dtype)
SHAPES = [
    (1000, 640, 64, 256, "bfloat16"),    # partial last block (1000 = 3 x 256 + 232), 1024 blocks
    (2048, 2048, 64, 40, "bfloat16"),    # 320 blocks: some workgroups take two, others one
    (512, 1152, 128, 128, "bfloat16"),   # d = 128: 256 blocks, 18 key tiles (Q prefetch needs 17)
    (768, 1088, 128, 96, "float16"),     # f16, 288 blocks
    (4096, 4096, 64, 16, "float16"),     # f16, 256 blocks of 64 tiles
    (1000, 1088, 128, 256, "bfloat16"),  # d = 128, partial last block, 1024 blocks (4 per workgroup)
]


@pytest.mark.parametrize("N,Nk,d,B,dtype", SHAPES)
def test_p4_bitwise_vs_8wave_and_oracle(fa, N, Nk, d, B, dtype):
    dt = torch.bfloat16 if dtype == "bfloat16" else torch.float16
    rng = np.random.default_rng(N + Nk + d + B)
    cast = lambda a: torch.tensor(a).to(dt)
    q, k, v = (rng.standard_normal(sh) for sh in ((N, d, B), (Nk, d, B), (Nk, d, B)))
    Q, K, V = (fa.jl_tensor(cast(a).double().numpy(), dt) for a in (q, k, v))
    y30, l30, m30, path30 = _run(fa, 30, Q, K, V)
    assert path30 == 30, "the shape meets the p4 launch rules, so variant 30 must run fa_fwd_p4"
    ref_variant = 7 if d <= 64 else 5
    y0, l0, m0, path0 = _run(fa, ref_variant, Q, K, V)
    assert path0 == 0
    assert torch.equal(y30.view(torch.int16), y0.view(torch.int16)), "y not bitwise equal to the 8-wave kernel"
    assert torch.equal(l30, l0) and torch.equal(m30, m0), "l, m not bitwise equal to the 8-wave kernel"
    # oracle on two slabs (the first and the last: different workgroups, streams crossing slabs)
    for b in (0, B - 1):
        qs, ks, vs = (cast(a[..., b:b + 1]).double().numpy() for a in (q, k, v))
        yr, lr, mr = O.dense_fa3(qs, ks, vs)
        assert_close(_np(y30[..., b:b + 1]), yr, dtype, f"y slab {b}")
        assert_lm_close(_np(l30[..., b:b + 1]), lr, dtype, f"l slab {b}")
        assert_lm_close(_np(m30[..., b:b + 1]), mr, dtype, f"m slab {b}")


@pytest.mark.parametrize("thr", [8.0, 0.0])
@pytest.mark.parametrize("d", [64, 128])
def test_p4_rescale_branch(fa, d, thr):
    """Running maxima that climb over the key sweep (every tile rescales at threshold
    0, most at threshold 8) plus spike keys, on 256 slabs: bitwise equal to the
    8-wave kernel at the same threshold, and within tolerance of the oracle."""
    L = fa.lib()
    rng = np.random.default_rng(23 + d)
    N, Nk, B = 256, 1152, 256
    u = rng.standard_normal(d); u /= np.linalg.norm(u)
    q = np.repeat((u * 6.0)[None, :, None], N, 0).repeat(B, 2) + 0.3 * rng.standard_normal((N, d, B))
    t = np.linspace(-1.0, 1.0, Nk) * 24.0
    k = t[:, None, None] * u[None, :, None] + 0.3 * rng.standard_normal((Nk, d, B))
    k[700] = q[10] * 5.0
    k[1100, :, 3] = q[200, :, 3] * 7.0
    v = rng.uniform(-4, 4, (Nk, d, B))
    bf = lambda a: torch.tensor(a).to(torch.bfloat16).double().numpy()
    q, k, v = bf(q), bf(k), bf(v)
    Q, K, V = (fa.jl_tensor(a, torch.bfloat16) for a in (q, k, v))
    old = L.fa_debug_set_rescale_threshold(thr)
    try:
        y30, l30, m30, path30 = _run(fa, 30, Q, K, V)
        y0, l0, m0, _ = _run(fa, 7 if d <= 64 else 5, Q, K, V)
    finally:
        L.fa_debug_set_rescale_threshold(old)
    assert path30 == 30
    assert torch.equal(y30.view(torch.int16), y0.view(torch.int16)), "y not bitwise equal"
    assert torch.equal(l30, l0) and torch.equal(m30, m0), "l, m not bitwise equal"
    for b in (0, 3):
        yr, lr, mr = O.dense_fa3(q[..., b:b + 1], k[..., b:b + 1], v[..., b:b + 1])
        assert_close(_np(y30[..., b:b + 1]), yr, "bfloat16", f"y slab {b}")
        assert_lm_close(_np(l30[..., b:b + 1]), lr, "bfloat16", f"l slab {b}")
        assert_lm_close(_np(m30[..., b:b + 1]), mr, "bfloat16", f"m slab {b}")


def test_p4_falls_back_outside_its_rules(fa):
    """Shapes outside the p4 rules (ragged key tiles, too few blocks for the grid,
    too few key tiles for the Q prefetch) run the 8-wave kernels under variant 30."""
    rng = np.random.default_rng(5)
    for (N, Nk, d, B) in ((1024, 1000, 64, 128), (256, 1024, 64, 8), (512, 512, 128, 128)):
        Q, K, V = (fa.jl_tensor(rng.standard_normal(sh), torch.bfloat16)
                   for sh in ((N, d, B), (Nk, d, B), (Nk, d, B)))
        y30, l30, m30, path30 = _run(fa, 30, Q, K, V)
        assert path30 == 0, (N, Nk, d, B)
        y0, l0, m0, _ = _run(fa, 0, Q, K, V)
        assert torch.equal(y30, y0) and torch.equal(l30, l0) and torch.equal(m30, m0)


def test_p4_is_the_d128_default(fa):
    """At d = dv = 128 the default forward (variant 0) runs fa_fwd_p4 on eligible shapes
    and equals the 8-wave kernel (variant 5) bitwise; at d = 64 the default stays the
    8-wave kernel."""
    rng = np.random.default_rng(77)
    for (N, d, B, want) in ((2048, 128, 64, 30), (2048, 64, 64, 0)):
        Q, K, V = (fa.jl_tensor(rng.standard_normal((N, d, B)), torch.bfloat16) for _ in range(3))
        y0, l0, m0, path0 = _run(fa, 0, Q, K, V)
        assert path0 == want, (d, path0)
        y5, l5, m5, _ = _run(fa, 5 if d == 128 else 7, Q, K, V)
        assert torch.equal(y0.view(torch.int16), y5.view(torch.int16))
        assert torch.equal(l0, l5) and torch.equal(m0, m5)
