"""GPU parity tests of the Float64 path (FA_DTYPE_F64) through the C ABI.

Float64 is the element type the reference tests and times in
(test/test.jl:12, logs/compare1.txt), so these tests hold the device to the
reference's own criterion there: Julia's `≈` at Float64, i.e.
norm(x − y) ≤ √eps(Float64)·max(norm(x), norm(y)), plus an elementwise bound of
1e-12·max|y| against the float64 oracle (oracle/fa_oracle.py).  l and m leave
the ABI as float32 for every dtype, so they are held to float32 rounding (1e-6
relative).  Inputs: the committed golden vectors and seeded random arrays.  The
golden files store their outputs as float32, so a golden case is checked against
the oracle re-run in float64 on the golden inputs (the fixture the 16/32-bit tests
read) and against the stored outputs at float32 rounding (G32)."""
from __future__ import annotations

import math

import numpy as np
import pytest
import torch

from conftest import golden_files, load_golden
from oracle import fa_oracle as O

pytestmark = pytest.mark.gpu

F64 = torch.float64
EPS64 = np.finfo(np.float64).eps
ELEM = 1e-12      # elementwise, relative to max(|y|, 1)
LM = 1e-6         # l, m: float32 outputs
G32 = 1e-6        # vs the float32-stored golden outputs, relative to max(|y|, 1)


@pytest.fixture(scope="module")
def fa():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm device")
    import fa_hip
    fa_hip.lib()
    return fa_hip


def _np(t):
    return t.detach().double().cpu().numpy()


def close64(x, y, what, nan_ok=False):
    x = np.asarray(x, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    assert x.shape == y.shape, f"{what}: shape {x.shape} vs {y.shape}"
    if nan_ok:
        nx, ny = np.isnan(x), np.isnan(y)
        assert np.array_equal(nx, ny), f"{what}: NaN pattern differs"
        x, y = x[~nx], y[~ny]
    assert np.all(np.isfinite(x)), f"{what}: non-finite values"
    if x.size == 0:
        return
    nrm = np.linalg.norm(x - y)
    assert nrm <= math.sqrt(EPS64) * max(np.linalg.norm(x), np.linalg.norm(y)), f"{what}: norm err {nrm:.3e}"
    err = np.abs(x - y).max() / max(np.abs(y).max(), 1.0)
    assert err <= ELEM, f"{what}: elementwise err {err:.3e}"


def vs_stored(x, y, what):
    x = np.asarray(x, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    ok = ~np.isnan(y)
    assert np.array_equal(np.isnan(x), ~ok), f"{what}: NaN pattern differs"
    err = np.abs(x[ok] - y[ok]).max() / max(np.abs(y[ok]).max(), 1.0) if ok.any() else 0.0
    assert err <= G32, f"{what} vs stored golden: {err:.3e}"


def lm64(x, y, what):
    x = np.asarray(x, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    err = np.abs(x - y).max() / max(np.abs(y).max(), 1e-30)
    assert err <= LM, f"{what}: {err:.3e}"


@pytest.mark.parametrize("path", golden_files("dense_"), ids=lambda p: p.split("/")[-1][:-4])
def test_dense_golden_f64(fa, path):
    g = load_golden(path)
    q, k, v = (fa.jl_tensor(g[x], F64) for x in ("q", "k", "v"))
    y, l, m = fa.dense_fa(q, k, v)
    torch.cuda.synchronize()
    assert y.dtype == F64 and tuple(y.shape) == g["y"].shape
    yr, lr, mr = O.dense_fa(g["q"], g["k"], g["v"])
    close64(_np(y), yr, "y")
    vs_stored(_np(y), g["y"], "y")
    lm64(_np(l), g["l"], "l")
    lm64(_np(m), g["m"], "m")


def test_reference_test_jl_in_float64(fa):
    """test/test.jl:5-21 as the reference runs it (Float64, Nq = Nkv = 30,
    dqk = 12, dv = 6, batch 2): dense_fa ≈ dense_dpa with Julia's Float64 `≈`."""
    rng = np.random.default_rng(0)
    q, k, v = rng.random((30, 12, 2)), rng.random((30, 12, 2)), rng.random((30, 6, 2))
    y, l, m = fa.dense_fa(*(fa.jl_tensor(a, F64) for a in (q, k, v)))
    y1, _ = O.dense_dpa(q, k, v)
    torch.cuda.synchronize()
    assert np.linalg.norm(_np(y) - y1) <= math.sqrt(EPS64) * np.linalg.norm(y1)
    close64(_np(y), y1, "dense_fa vs dense_dpa")
    # and the device's own materialising dense_dpa (library GEMMs + fa_softmax)
    yd, _ = fa.dense_dpa(*(fa.jl_tensor(a, F64) for a in (q, k, v)))
    torch.cuda.synchronize()
    close64(_np(yd), y1, "device dense_dpa")


@pytest.mark.parametrize("N,Nk,d,dv,B", [(1, 1, 64, 64, 1), (1, 300, 64, 64, 2), (300, 1, 64, 64, 2),
                                         (65, 63, 16, 8, 2), (129, 257, 128, 128, 1), (127, 65, 128, 32, 2),
                                         (33, 4100, 64, 64, 1), (3, 7, 1, 1, 2), (70, 70, 33, 65, 1),
                                         (512, 512, 64, 64, 4)])
def test_dense_shapes_f64(fa, N, Nk, d, dv, B):
    rng = np.random.default_rng(N * 1000 + Nk)
    q, k, v = rng.standard_normal((N, d, B)), rng.standard_normal((Nk, d, B)), rng.standard_normal((Nk, dv, B))
    y, l, m = fa.dense_fa(*(fa.jl_tensor(a, F64) for a in (q, k, v)))
    yr, lr, mr = O.dense_fa3(q, k, v)
    torch.cuda.synchronize()
    close64(_np(y), yr, "y")
    lm64(_np(l), lr, "l")
    lm64(_np(m), mr, "m")


def test_dense_f64_spiky_scores(fa):
    """Scores spanning hundreds of natural-log units: the online max must keep
    every exponential in range (src/dense.jl:78-91) in double as well."""
    rng = np.random.default_rng(3)
    N, d, B = 200, 32, 2
    q = rng.standard_normal((N, d, B)) * 4.0
    k = rng.standard_normal((N, d, B)) * 4.0
    v = rng.standard_normal((N, d, B))
    k[150] = q[10] * 5.0
    y, l, m = fa.dense_fa(*(fa.jl_tensor(a, F64) for a in (q, k, v)))
    yr, lr, mr = O.dense_fa3(q, k, v)
    torch.cuda.synchronize()
    close64(_np(y), yr, "y")
    lm64(_np(m), mr, "m")


def test_dense_f64_explicit_scale(fa):
    rng = np.random.default_rng(4)
    q, k, v = (rng.standard_normal((96, 16, 2)) for _ in range(3))
    y, _, _ = fa.dense_fa(*(fa.jl_tensor(a, F64) for a in (q, k, v)), scale=0.5)
    s = np.einsum("nfb,kfb->bnk", q, k) * 0.5
    p = np.exp(s - s.max(-1, keepdims=True))
    p /= p.sum(-1, keepdims=True)
    yr = np.einsum("bnk,kcb->ncb", p, v)
    torch.cuda.synchronize()
    close64(_np(y), yr, "y")


def _grad_close(x, y, what):
    close64(x, y, what)


@pytest.mark.parametrize("path", golden_files("bwd_"), ids=lambda p: p.split("/")[-1][:-4])
def test_backward_golden_f64(fa, path):
    g = load_golden(path)
    Q, K, V, dO = (fa.jl_tensor(g[x], F64) for x in ("q", "k", "v", "do"))
    Oo, l, m = fa.dense_fa(Q, K, V)
    dQ, dK, dV = fa.dense_fa_backward(Q, K, V, Oo, dO, l, m)
    torch.cuda.synchronize()
    assert dQ.dtype == F64
    o, lr, mr = O.dense_fa3(g["q"], g["k"], g["v"])
    ref = O.dense_fa_backward(g["q"], g["k"], g["v"], o, g["do"], lr, mr)
    for x, r, nm in zip((dQ, dK, dV), ref, ("dq", "dk", "dv")):
        _grad_close(_np(x), r, nm)
        vs_stored(_np(x), g[nm], nm)


@pytest.mark.parametrize("N,Nk,d,dv,B", [(64, 64, 64, 64, 2), (256, 192, 128, 128, 2), (100, 77, 12, 6, 3),
                                         (1, 5, 16, 16, 1), (130, 1, 32, 8, 2), (200, 320, 64, 128, 2),
                                         (72, 1000, 128, 32, 1)])
def test_backward_vs_oracle_f64(fa, N, Nk, d, dv, B):
    rng = np.random.default_rng(N * 31 + Nk)
    q, k = rng.standard_normal((N, d, B)), rng.standard_normal((Nk, d, B))
    v, do = rng.standard_normal((Nk, dv, B)), rng.standard_normal((N, dv, B))
    Q, K, V, dO = (fa.jl_tensor(a, F64) for a in (q, k, v, do))
    Oo, l, m = fa.dense_fa(Q, K, V)
    dQ, dK, dV = fa.dense_fa_backward(Q, K, V, Oo, dO, l, m)
    o, lr, mr = O.dense_fa3(q, k, v)
    dq, dk, dv_ = O.dense_fa_backward(q, k, v, o, do, lr, mr)
    torch.cuda.synchronize()
    _grad_close(_np(dQ), dq, "dQ")
    _grad_close(_np(dK), dk, "dK")
    _grad_close(_np(dV), dv_, "dV")


def test_backward_f64_matches_autograd(fa):
    """Independent of the oracle: torch autograd of the materialised attention in
    float64 on the host."""
    rng = np.random.default_rng(11)
    N, Nk, d, dv, B = 90, 110, 24, 20, 2
    q, k = rng.standard_normal((N, d, B)), rng.standard_normal((Nk, d, B))
    v, do = rng.standard_normal((Nk, dv, B)), rng.standard_normal((N, dv, B))
    Q, K, V, dO = (fa.jl_tensor(a, F64) for a in (q, k, v, do))
    Oo, l, m = fa.dense_fa(Q, K, V)
    dQ, dK, dV = fa.dense_fa_backward(Q, K, V, Oo, dO, l, m)
    qt, kt, vt = (torch.tensor(a, requires_grad=True) for a in (q, k, v))
    s = torch.einsum("nfb,kfb->bnk", qt, kt) / math.sqrt(d)
    y = torch.einsum("bnk,kcb->ncb", torch.softmax(s, -1), vt)
    y.backward(torch.tensor(do))
    torch.cuda.synchronize()
    close64(_np(Oo), y.detach().numpy(), "O")
    _grad_close(_np(dQ), qt.grad.numpy(), "dQ")
    _grad_close(_np(dK), kt.grad.numpy(), "dK")
    _grad_close(_np(dV), vt.grad.numpy(), "dV")


def test_backward_f64_empty(fa):
    Q = fa.jl_tensor(np.ones((4, 8, 1)), F64)
    K = fa.jl_empty((0, 8, 1), F64)
    V = fa.jl_empty((0, 8, 1), F64)
    Oo, l, m = fa.dense_fa(Q, K, V)
    torch.cuda.synchronize()
    assert torch.all(Oo == 0) and torch.all(l == 0) and torch.all(torch.isinf(m))
    dQ, dK, dV = fa.dense_fa_backward(Q, K, V, Oo, fa.jl_tensor(np.ones((4, 8, 1)), F64), l, m)
    torch.cuda.synchronize()
    assert torch.all(dQ == 0) and dK.numel() == 0 and dV.numel() == 0


@pytest.mark.parametrize("path", golden_files("wind_") + golden_files("block_"),
                         ids=lambda p: p.split("/")[-1][:-4])
def test_windowed_golden_f64(fa, path):
    g = load_golden(path)
    ws, st, pad = int(g["ws"]), int(g["stride"]), int(g["pad"])
    q, k, v, dy = (fa.jl_tensor(g[x], F64) for x in ("q", "k", "v", "dy"))
    y, l, m = fa.windowed_fa(q, k, v, ws, stride=st, pad=pad)
    dq, dk, dv = fa.windowed_fa_backward(q, k, v, y, dy, l, m, ws, stride=st, pad=pad)
    torch.cuda.synchronize()
    yr, _, _ = O.windowed_fa(g["q"], g["k"], g["v"], ws, st, pad)
    close64(_np(y), yr, "y", nan_ok=True)
    vs_stored(_np(y), g["y"], "y")
    lm64(_np(l), g["l"], "l")
    lm64(_np(m), g["m"], "m")
    ref = O.windowed_fa_backward(g["q"], g["k"], g["v"], g["dy"], ws, st, pad)
    for x, r, nm in zip((dq, dk, dv), ref, ("dq", "dk", "dv")):
        close64(_np(x), r, nm)
        vs_stored(_np(x), g[nm], nm)


def test_windowed_config3_shape_f64(fa):
    """configs[2]'s geometry (128x128, ws 7, d 64) at B = 1 in Float64 vs the oracle."""
    rng = np.random.default_rng(12)
    q, k, v = (rng.standard_normal((128, 128, 64, 1)) for _ in range(3))
    y, l, m = fa.windowed_fa(*(fa.jl_tensor(a, F64) for a in (q, k, v)), 7)
    yr, lr, mr = O.windowed_fa(q, k, v, 7)
    torch.cuda.synchronize()
    close64(_np(y), yr, "y", nan_ok=True)
    lm64(_np(m), mr, "m")


def test_window_unwindow_f64(fa):
    rng = np.random.default_rng(13)
    x = rng.standard_normal((13, 11, 5, 2))
    for ws, st, pad in ((3, 1, 1), (4, 2, 0), (5, 5, 2)):
        X = fa.window(fa.jl_tensor(x, F64), ws, st, pad)
        Xr = O.window(x, ws, st, pad)
        torch.cuda.synchronize()
        assert np.array_equal(_np(X), Xr), (ws, st, pad)   # a pure gather: bit-exact
        xb = fa.unwindow(X, x.shape, ws, st, pad)
        xr = O.unwindow(Xr, x.shape, ws, st, pad)
        torch.cuda.synchronize()
        close64(_np(xb), xr, f"unwindow {(ws, st, pad)}")


@pytest.mark.parametrize("path", golden_files("circ_"), ids=lambda p: p.split("/")[-1][:-4])
def test_circulant_golden_f64(fa, path):
    g = load_golden(path)
    Q, K, V = (fa.jl_tensor(g[x], F64) for x in ("q", "k", "v"))
    o, l, m = fa.circulant_fa(Q, K, V, int(g["W"]))
    torch.cuda.synchronize()
    orf, _, _ = O.circulant_fa3(g["q"], g["k"], g["v"], int(g["W"]))
    close64(_np(o), orf, "O")
    vs_stored(_np(o), g["o"], "O")
    lm64(_np(l), g["l"], "l")
    lm64(_np(m), g["m"], "m")


@pytest.mark.parametrize("N,d,dv,W,B", [(512, 64, 64, 129, 2), (96, 64, 32, 200, 1), (1001, 32, 16, 33, 2),
                                        (640, 64, 64, 2, 1)])
def test_circulant_f64(fa, N, d, dv, W, B):
    rng = np.random.default_rng(N + W)
    q, k, v = rng.standard_normal((N, d, B)), rng.standard_normal((N, d, B)), rng.standard_normal((N, dv, B))
    o, l, m = fa.circulant_fa(*(fa.jl_tensor(a, F64) for a in (q, k, v)), W)
    orf, lr, mr = O.circulant_fa3(q, k, v, W)
    torch.cuda.synchronize()
    close64(_np(o), orf, "O")
    lm64(_np(m), mr, "m")


@pytest.mark.parametrize("path", golden_files("softmax_"), ids=lambda p: p.split("/")[-1][:-4])
def test_softmax_golden_f64(fa, path):
    g = load_golden(path)
    P = fa.fused_softmax(fa.jl_tensor(g["s"], F64), int(g["dims"]))
    torch.cuda.synchronize()
    close64(_np(P), O.fused_softmax(g["s"], int(g["dims"])), "P", nan_ok=True)
    vs_stored(_np(P), g["p"], "P")


@pytest.mark.parametrize("shape,dims", [((4096, 64, 3), 1), ((50000, 3, 2), 1), ((1000, 32, 2), 2),
                                        ((777, 129, 3), 2), ((100000,), 1)])
def test_softmax_f64(fa, shape, dims):
    rng = np.random.default_rng(len(shape) * 7 + dims)
    s = rng.standard_normal(shape) * 8.0
    P = fa.fused_softmax(fa.jl_tensor(s, F64), dims)
    torch.cuda.synchronize()
    close64(_np(P), O.fused_softmax(s, dims), "P")


def test_softmax_f64_special_values(fa):
    """All −Inf → NaN, a +Inf entry → NaN (the reference's arithmetic)."""
    s = np.zeros((4, 3))
    s[:, 0] = -np.inf
    s[1, 1] = np.inf
    P = _np(fa.fused_softmax(fa.jl_tensor(s, F64), 1))
    torch.cuda.synchronize()
    assert np.all(np.isnan(P[:, 0])) and np.all(np.isnan(P[:, 1]))
    close64(P[:, 2], np.full(4, 0.25), "uniform column")


@pytest.mark.parametrize("W", [16, 128])
def test_reference_runwindow_case_f64(fa, W):
    """bench/compare.jl:32-57 / :105-115 (runwindow: N = 4096, d = 32, bs = 1,
    stride 8, pad 0, Float64): the reference asserts windowed_dpa ≈ windowed_fa
    at its own benchmark shape; here the device windowed_fa against the oracle and
    against the device's materialising windowed_dpa, at Float64 `≈`."""
    rng = np.random.default_rng(W)
    q, k, v = (rng.standard_normal((4096, 32, 1)) for _ in range(3))
    Q, K, V = (fa.jl_tensor(a, F64) for a in (q, k, v))
    y, l, m = fa.windowed_fa(Q, K, V, W, stride=8, pad=0)
    yd, _ = fa.windowed_dpa(Q, K, V, W, 8, 0)
    yr, _, _ = O.windowed_fa(q, k, v, W, 8, 0)
    torch.cuda.synchronize()
    close64(_np(y), yr, "windowed_fa vs oracle", nan_ok=True)
    close64(_np(yd), _np(y), "windowed_dpa vs windowed_fa", nan_ok=True)


@pytest.mark.parametrize("N,W", [(4096, 16), (4096, 129), (300, 301)])
def test_circulant_dpa_f64(fa, N, W):
    """circulant_dpa ≈ circulant_fa at Float64 (bench/compare.jl:72-74, the
    reference's runcirculant shape N = 4096, d = 32) and both vs the oracle."""
    rng = np.random.default_rng(W)
    q, k, v = (rng.standard_normal((N, 32, 1)) for _ in range(3))
    Q, K, V = (fa.jl_tensor(a, F64) for a in (q, k, v))
    o, P = fa.circulant_dpa(Q, K, V, W)
    of, _, _ = fa.circulant_fa(Q, K, V, W)
    orf, Pr = O.circulant_dpa3(q, k, v, W)
    torch.cuda.synchronize()
    close64(_np(o), orf, "O")
    close64(_np(P), Pr, "P")
    close64(_np(of), _np(o), "circulant_fa vs circulant_dpa")
