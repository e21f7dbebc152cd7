"""GPU parity tests: circulant (periodic banded) attention through the C ABI
(fa_circulant_fwd) vs the float64 oracle restatement of circulant_fa!
(src/circulant.jl:9-118) on the committed golden vectors, on both kernels
(tiled MFMA path: bf16/fp16 with N % 8 == 0; generic path: fp32, ragged N),
band edge cases (W = 1, even W, W > N) and a full-size property check against
a float32 torch band gather.  Tolerances: tests/conftest.py."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from conftest import assert_close, assert_lm_close, golden_files, load_golden
from oracle import fa_oracle as O

pytestmark = pytest.mark.gpu

DT = {"float32": torch.float32, "bfloat16": torch.bfloat16, "float16": torch.float16}


@pytest.fixture(scope="module")
def fa():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm device")
    import fa_hip
    fa_hip.lib()
    return fa_hip


def _np(t):
    return t.detach().float().cpu().numpy().astype(np.float64)


def _round(a, dtype):
    """Inputs as the device sees them (so the oracle runs on identical values)."""
    return torch.tensor(a).to(DT[dtype]).double().numpy()


@pytest.mark.parametrize("dtype", list(DT))
@pytest.mark.parametrize("path", golden_files("circ_"), ids=lambda p: p.split("/")[-1][:-4])
def test_circulant_golden(fa, path, dtype):
    g = load_golden(path)
    Q, K, V = (fa.jl_tensor(g[x], DT[dtype]) for x in ("q", "k", "v"))
    o, l, m = fa.circulant_fa(Q, K, V, int(g["W"]))
    torch.cuda.synchronize()
    assert fa.is_jl_contiguous(o) and tuple(o.shape) == g["o"].shape
    assert_close(_np(o), g["o"], dtype, "O")
    assert_lm_close(_np(l), g["l"], dtype, "l")
    assert_lm_close(_np(m), g["m"], dtype, "m")


CASES = [
    # N, d, dv, W, B
    (512, 64, 64, 129, 2),      # reference bench window (128 + 1), several workgroups
    (4096, 32, 32, 256, 1),     # runcirculant's largest window (bench/compare.jl:105)
    (1024, 128, 128, 511, 1),   # wide band, d = 128
    (96, 64, 32, 200, 1),       # W > N on the tiled path
    (1001, 32, 16, 33, 2),      # ragged N: generic path for every dtype
    (640, 64, 64, 2, 1),        # even, tiny W: most tiles masked
]


@pytest.mark.parametrize("dtype", ["bfloat16", "float16", "float32"])
@pytest.mark.parametrize("N,d,dv,W,B", CASES)
def test_circulant_random(fa, N, d, dv, W, B, dtype):
    rng = np.random.default_rng(N * 7 + W)
    Qh, Kh, Vh = rng.standard_normal((N, d, B)), rng.standard_normal((N, d, B)), rng.standard_normal((N, dv, B))
    Qh, Kh, Vh = (_round(a, dtype) for a in (Qh, Kh, Vh))
    o, l, m = fa.circulant_fa(*(fa.jl_tensor(a, DT[dtype]) for a in (Qh, Kh, Vh)), W)
    torch.cuda.synchronize()
    Oo, lo, mo = O.circulant_fa3(Qh, Kh, Vh, W)
    assert_close(_np(o), Oo, dtype, "O")
    assert_lm_close(_np(l), lo, dtype, "l")
    assert_lm_close(_np(m), mo, dtype, "m")


def test_circulant_scale_and_inplace(fa):
    """Explicit scale (<= 0 means 1/√d); in-place form overwrites every output."""
    rng = np.random.default_rng(3)
    N, d, W = 256, 64, 31
    Qh, Kh, Vh = (_round(rng.standard_normal((N, d, 1)), "bfloat16") for _ in range(3))
    Q, K, V = (fa.jl_tensor(a, torch.bfloat16) for a in (Qh, Kh, Vh))
    o = fa.jl_tensor(np.full((N, d, 1), 7.0), torch.bfloat16)
    l = fa.jl_tensor(np.full((N, 1, 1), -3.0), torch.float32)
    m = fa.jl_tensor(np.full((N, 1, 1), 99.0), torch.float32)
    fa.circulant_fa_(o, l, m, Q, K, V, W, scale=0.05)
    torch.cuda.synchronize()
    # oracle with scale 0.05 = pre-scaling Q by 0.05·√d under τ = 1/√d
    Oo, lo, mo = O.circulant_fa3(Qh * 0.05 * np.sqrt(d), Kh, Vh, W)
    assert_close(_np(o), Oo, "bfloat16", "O")
    assert_lm_close(_np(l), lo, "bfloat16", "l")
    assert_lm_close(_np(m), mo, "bfloat16", "m")


def test_circulant_deterministic(fa):
    rng = np.random.default_rng(4)
    Q, K, V = (fa.jl_tensor(rng.standard_normal((2048, 64, 2)), torch.bfloat16) for _ in range(3))
    a = fa.circulant_fa(Q, K, V, 129)
    b = fa.circulant_fa(Q, K, V, 129)
    torch.cuda.synchronize()
    for x, y in zip(a, b):
        assert torch.equal(x, y)


def test_circulant_full_size_band_property(fa):
    """(B·H, N, d, W) = (64, 16384, 64, 129) bf16: two slabs against a float32
    torch band gather of the same bf16 inputs; softmax weights sum to one."""
    N, d, B, W = 16384, 64, 64, 129
    g = torch.Generator(device="cuda").manual_seed(5)
    Q, K, V = (fa.jl_empty((N, d, B), torch.bfloat16) for _ in range(3))
    for t in (Q, K, V):
        t.copy_(torch.randn((N, d, B), generator=g, device="cuda"))
    o, l, m = fa.circulant_fa(Q, K, V, W)
    torch.cuda.synchronize()
    p = (W - 1) // 2
    idx = (torch.arange(N, device="cuda")[:, None] - p + torch.arange(W, device="cuda")[None, :]) % N
    for b in (0, B - 1):
        q, k, v = (x[:, :, b].float() for x in (Q, K, V))
        s = torch.einsum("nd,nwd->nw", q, k[idx]) / d ** 0.5
        mm = s.max(dim=1).values
        e = torch.exp(s - mm[:, None])
        ll = e.sum(dim=1)
        ref = torch.einsum("nw,nwc->nc", e / ll[:, None], v[idx])
        assert_close(o[:, :, b].float().cpu().numpy(), ref.cpu().numpy().astype(np.float64), "bfloat16", f"O[{b}]")
        assert torch.allclose(m[:, 0, b], mm, rtol=1e-4, atol=1e-4)
        assert torch.allclose(l[:, 0, b], ll, rtol=1e-4)
    assert torch.isfinite(o.float()).all()


@pytest.mark.parametrize("N,d,dv,W,dtype", [(100, 32, 16, 9, "float32"), (257, 64, 64, 129, "bfloat16"),
                                            (30, 12, 6, 7, "float16"), (64, 128, 96, 65, "float32"),
                                            (1000, 64, 32, 1001, "bfloat16"), (5, 8, 8, 12, "float32")])
def test_circulant_simt_vs_reference_kernel(fa, N, d, dv, W, dtype):
    """The LDS-tiled SIMT kernel (fp32 / ragged N) against the oracle and
    against the one-wave-per-query reference kernel on the same inputs."""
    tdt = {"float32": torch.float32, "bfloat16": torch.bfloat16, "float16": torch.float16}[dtype]
    rng = np.random.default_rng(N + W + d)
    cast = lambda a: torch.tensor(a).to(tdt).double().numpy()
    q, k = cast(rng.standard_normal((N, d, 2))), cast(rng.standard_normal((N, d, 2)))
    v = cast(rng.standard_normal((N, dv, 2)))
    Q, K, V = (fa.jl_tensor(a, tdt) for a in (q, k, v))
    L = fa.lib()
    L.fa_debug_set_circ_generic(2)          # force the SIMT kernel (small grids pick the other)
    try:
        o1, l1, m1 = fa.circulant_fa(Q, K, V, W)
    finally:
        L.fa_debug_set_circ_generic(0)
    L.fa_debug_set_circ_generic(1)
    try:
        o2, l2, m2 = fa.circulant_fa(Q, K, V, W)
    finally:
        L.fa_debug_set_circ_generic(0)
    torch.cuda.synchronize()
    orr, lr, mr = O.circulant_fa3(q, k, v, W)
    assert_close(_np(o1), orr, dtype, "O")
    assert_lm_close(_np(l1), lr, dtype, "l")
    assert_lm_close(_np(m1), mr, dtype, "m")
    assert_close(_np(o1), _np(o2), dtype, "O simt vs one-wave")


@pytest.mark.parametrize("dtype", list(DT))
@pytest.mark.parametrize("N,d,dv,W,B", [(96, 32, 16, 7, 2), (200, 64, 64, 65, 1), (50, 16, 8, 64, 2)])
def test_circulant_dpa_vs_oracle(fa, dtype, N, d, dv, W, B):
    """circulant_dpa (src/naive/circulant.jl:1-36): O and the (W, N, B) band P vs
    the oracle, and the reference's own check circulant_dpa ≈ circulant_fa
    (bench/compare.jl:72-74)."""
    rng = np.random.default_rng(N + W)
    rt = lambda a: torch.tensor(a).to(DT[dtype]).double().numpy()
    q, k, v = rt(rng.standard_normal((N, d, B))), rt(rng.standard_normal((N, d, B))), rt(rng.standard_normal((N, dv, B)))
    Q, K, V = (fa.jl_tensor(a, DT[dtype]) for a in (q, k, v))
    o, P = fa.circulant_dpa(Q, K, V, W)
    of, _, _ = fa.circulant_fa(Q, K, V, W)
    orf, Pr = O.circulant_dpa3(q, k, v, W)
    torch.cuda.synchronize()
    assert tuple(P.shape) == (W, N, B) and fa.is_jl_contiguous(P)
    assert_close(_np(o), orf, dtype, "O")
    assert_close(_np(P), Pr, dtype, "P")
    assert_close(_np(o), _np(of), dtype, "circulant_dpa vs circulant_fa")
