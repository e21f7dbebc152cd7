"""CPU tests of the oracle itself: pin the numpy restatement (oracle/fa_oracle.py)
to independent implementations present in this image (torch CPU sdpa,
autograd, F.unfold / F.fold), to the committed golden vectors, and to the C
port (oracle/fa_cpu.c).  No GPU needed."""
from __future__ import annotations

import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import golden_files, load_golden
from oracle import fa_oracle as O


def _sdpa(q, k, v):
    """torch reference on Julia-shaped (N, d, B) numpy arrays."""
    t = lambda a: torch.tensor(np.asarray(a)).permute(2, 0, 1)
    return F.scaled_dot_product_attention(t(q), t(k), t(v)).permute(1, 2, 0).numpy()


def test_tile_policy_matches_reference():
    # src/dense.jl:34-35 with M = 32000; documented values in SURVEY.md §3
    assert O.tile_policy(4096, 64) == (64, 500)
    assert O.tile_policy(8192, 128) == (128, 250)
    assert O.tile_policy(30, 12) == (12, 30)          # Bc clamped to N
    assert O.tile_policy(512, 64) == (64, 500)


@pytest.mark.parametrize("N,Nk,d,dv,B,M", [(30, 30, 12, 6, 2, 32000), (70, 53, 12, 6, 3, 100),
                                           (257, 257, 64, 64, 2, 32000), (130, 200, 32, 48, 1, 500)])
def test_dense_fa_vs_dpa_vs_torch(N, Nk, d, dv, B, M):
    rng = np.random.default_rng(N + Nk)
    q, k, v = rng.standard_normal((N, d, B)), rng.standard_normal((Nk, d, B)), rng.standard_normal((Nk, dv, B))
    y1, P = O.dense_dpa(q, k, v)
    y2, l, m = O.dense_fa(q, k, v, M=M)
    assert np.allclose(y1, y2, atol=1e-12)
    assert np.allclose(y1, _sdpa(q, k, v), atol=1e-12)
    s = np.einsum("nkb,jkb->njb", q, k) / math.sqrt(d)
    assert np.allclose(m[:, 0], s.max(1), atol=1e-12)
    assert np.allclose(l[:, 0], np.exp(s - s.max(1, keepdims=True)).sum(1), rtol=1e-12)
    assert np.allclose(P.sum(1), 1.0)


def test_nd_wrapper_flattens_spatial_column_major():
    rng = np.random.default_rng(3)
    q = rng.standard_normal((5, 4, 8, 2))
    y, l, m = O.dense_fa(q, q, q)
    Q = np.reshape(q, (20, 8, 2), order="F")
    y3, l3, m3 = O.dense_fa3(Q, Q, Q)
    assert np.allclose(np.reshape(y, (20, 8, 2), order="F"), y3)
    assert l.shape == (20, 1, 2)


@pytest.mark.parametrize("N,Nk,d,dv,B", [(64, 64, 16, 16, 2), (45, 77, 12, 6, 2), (300, 280, 32, 20, 1)])
def test_backward_vs_autograd(N, Nk, d, dv, B):
    rng = np.random.default_rng(N * 7 + Nk)
    q, k, v = rng.standard_normal((N, d, B)), rng.standard_normal((Nk, d, B)), rng.standard_normal((Nk, dv, B))
    dO = rng.standard_normal((N, dv, B))
    Oo, l, m = O.dense_fa3(q, k, v, M=600)
    dq, dk, dvv = O.dense_fa_backward(q, k, v, Oo, dO, l, m, M=600)
    tq, tk, tv = (torch.tensor(a).permute(2, 0, 1).requires_grad_() for a in (q, k, v))
    F.scaled_dot_product_attention(tq, tk, tv).backward(torch.tensor(dO).permute(2, 0, 1))
    g = lambda t: t.grad.permute(1, 2, 0).numpy()
    assert np.allclose(dq, g(tq), atol=1e-11)
    assert np.allclose(dk, g(tk), atol=1e-11)
    assert np.allclose(dvv, g(tv), atol=1e-11)


@pytest.mark.parametrize("ws,st,pad", [(3, 3, 1), (3, 2, 1), (7, 7, 3), (4, 3, 0), (5, 1, 2), (2, 3, 0)])
def test_window_unwindow_match_torch_unfold_fold(ws, st, pad):
    # Julia (S1=W, S2=H, C, B) column-major == torch (B, C, H, W) row-major.
    rng = np.random.default_rng(ws * 10 + st)
    W, H, C, B = 13, 11, 3, 2
    x = rng.standard_normal((W, H, C, B))
    X = O.window(x, ws, st, pad)
    tx = torch.tensor(x).permute(3, 2, 1, 0)
    U = F.unfold(tx, ws, padding=pad, stride=st).numpy()
    T, Cc, L, Bb = X.shape
    assert np.array_equal(X.transpose(3, 1, 0, 2).reshape(B, C * T, L), U)
    y = O.unwindow(X, (W, H, C, B), ws, st, pad)
    Fd = F.fold(torch.tensor(U), (H, W), ws, padding=pad, stride=st).permute(3, 2, 1, 0).numpy()
    assert np.allclose(y, Fd, atol=1e-12)


def test_window_1d_and_3d_adjointness():
    rng = np.random.default_rng(5)
    for shape, ws, st, pad in [((17, 3, 2), 5, 2, 2), ((6, 5, 4, 2, 1), 3, 2, 1)]:
        x = rng.standard_normal(shape)
        X = O.window(x, ws, st, pad)
        Y = rng.standard_normal(X.shape)
        # <window(x), Y> == <x, unwindow(Y)>  (fold is the adjoint of unfold)
        assert np.isclose(np.sum(X * Y), np.sum(x * O.unwindow(Y, shape, ws, st, pad)))


def test_windowed_fa_equals_windowed_dpa_and_nan_tail():
    rng = np.random.default_rng(6)
    q = rng.standard_normal((64, 4, 1))
    y, lw, mw = O.windowed_fa(q, q, q, 64)        # pad 31: pixels 33..63 uncovered → NaN (Appendix A.7)
    assert np.isnan(y[33:]).all() and not np.isnan(y[:33]).any()
    assert lw.shape == (64, 1, 1, 1)
    x = rng.standard_normal((10, 9, 4, 2))
    y1, _, _ = O.windowed_fa(x, x, x, 3, 2, 1)
    y2 = O.windowed_dpa(x, x, x, 3, 2, 1)
    assert np.allclose(y1, y2, atol=1e-12)


def test_windowed_backward_vs_autograd():
    rng = np.random.default_rng(8)
    W, H, C, B, ws, st, pad = 9, 8, 4, 2, 3, 2, 1
    q, k, v, dy = (rng.standard_normal((W, H, C, B)) for _ in range(4))
    dq, dk, dvv = O.windowed_fa_backward(q, k, v, dy, ws, st, pad)

    def tw(x):   # torch window: (B, C, H, W) -> (B*L, T, C)
        U = F.unfold(x, ws, padding=pad, stride=st)            # (B, C*T, L)
        Bn, CT, L = U.shape
        return U.reshape(Bn, C, ws * ws, L).permute(0, 3, 2, 1).reshape(Bn * L, ws * ws, C), L

    tq, tk, tv = (torch.tensor(a).permute(3, 2, 1, 0).requires_grad_() for a in (q, k, v))
    qw, L = tw(tq); kw, _ = tw(tk); vw, _ = tw(tv)
    yw = F.scaled_dot_product_attention(qw, kw, vw)            # (B*L, T, C)
    U = yw.reshape(B, L, ws * ws, C).permute(0, 3, 2, 1).reshape(B, C * ws * ws, L)
    ones = torch.ones(1, 1, H, W, dtype=torch.float64)
    div = F.fold(F.unfold(ones, ws, padding=pad, stride=st), (H, W), ws, padding=pad, stride=st)
    y = F.fold(U, (H, W), ws, padding=pad, stride=st) / div
    y.backward(torch.tensor(dy).permute(3, 2, 1, 0))
    g = lambda t: t.grad.permute(3, 2, 1, 0).numpy()
    assert np.allclose(dq, g(tq), atol=1e-11)
    assert np.allclose(dk, g(tk), atol=1e-11)
    assert np.allclose(dvv, g(tv), atol=1e-11)


@pytest.mark.parametrize("path", golden_files("dense_"))
def test_golden_dense_reproduces(path):
    g = load_golden(path)
    y, l, m = O.dense_fa(g["q"], g["k"], g["v"])
    assert np.allclose(y, g["y"], rtol=1e-6, atol=1e-6)
    assert np.allclose(l, g["l"], rtol=1e-12) and np.allclose(m, g["m"], rtol=1e-12, atol=1e-12)
    assert np.allclose(_sdpa(np.reshape(g["q"], (-1,) + g["q"].shape[-2:], order="F"),
                             np.reshape(g["k"], (-1,) + g["k"].shape[-2:], order="F"),
                             np.reshape(g["v"], (-1,) + g["v"].shape[-2:], order="F")),
                       np.reshape(g["y"], (-1,) + g["y"].shape[-2:], order="F"), atol=1e-5)


@pytest.mark.parametrize("path", golden_files("bwd_"))
def test_golden_backward_reproduces(path):
    g = load_golden(path)
    dq, dk, dv = O.dense_fa_backward(g["q"], g["k"], g["v"], g["o"], g["do"], g["l"], g["m"])
    for a, b in ((dq, g["dq"]), (dk, g["dk"]), (dv, g["dv"])):
        assert np.allclose(a, b, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("path", golden_files("wind_") + golden_files("block_"))
def test_golden_windowed_reproduces(path):
    g = load_golden(path)
    ws, st, pad = int(g["ws"]), int(g["stride"]), int(g["pad"])
    y, l, m = O.windowed_fa(g["q"], g["k"], g["v"], ws, st, pad)
    assert np.allclose(y, g["y"], atol=1e-6, equal_nan=True)
    assert np.allclose(l, g["l"]) and np.allclose(m, g["m"])
    dq, dk, dv = O.windowed_fa_backward(g["q"], g["k"], g["v"], g["dy"], ws, st, pad)
    assert np.allclose(dq, g["dq"], atol=1e-5) and np.allclose(dv, g["dv"], atol=1e-5)


@pytest.mark.parametrize("path", golden_files("dense_")[:4])
def test_cpu_port_matches_oracle(path):
    from oracle import cpu_port
    g = load_golden(path)
    D = g["q"].ndim
    r = lambda a: np.reshape(a, (-1,) + a.shape[-2:], order="F")
    O64, l64, m64 = cpu_port.dense_fa(r(g["q"]), r(g["k"]), r(g["v"]), nthreads=2)
    assert np.allclose(O64, r(g["y"]), atol=1e-6)
    assert np.allclose(l64, g["l"]) and np.allclose(m64, g["m"])
    O32, l32, m32 = cpu_port.dense_fa(r(g["q"]).astype(np.float32), r(g["k"]).astype(np.float32),
                                      r(g["v"]).astype(np.float32), nthreads=2)
    assert np.abs(O32 - r(g["y"])).max() < 1e-5
    assert D >= 3


# --- circulant (src/circulant.jl, src/naive/circulant.jl, src/utils.jl:4-17) ---
@pytest.mark.parametrize("N,W", [(10, 3), (10, 4), (30, 7), (20, 29), (64, 16), (5, 12), (9, 1)])
def test_cartesian_circulant_is_the_periodic_band(N, W):
    """cartesian_circulant enumerates, for column i, the band (i − p + t) mod N,
    t = 0..W−1 (with multiplicity when W > N); for odd W <= N (the reference's
    precondition, src/utils.jl:7) the circshift makes the rows come out sorted."""
    J = O.circulant_index(N, W)
    p = (W - 1) // 2
    for i in range(N):
        band = sorted((i - p + t) % N for t in range(W))
        assert sorted(J[:, i].tolist()) == band
        if W <= N and W % 2 == 1:
            assert list(J[:, i]) == sorted(J[:, i])      # CSC rowvals come out sorted


def _torch_band_sdpa(Q, K, V, W):
    """Independent restatement: dense SDPA with an additive band mask (torch CPU)."""
    N, d, B = Q.shape
    p = (W - 1) // 2
    out = np.zeros((N, V.shape[1], B))
    i = np.arange(N)[:, None]
    for b in range(B):
        # multiplicity: count how many band entries t hit key j
        cnt = np.zeros((N, N))
        for t in range(W):
            np.add.at(cnt, (np.arange(N), (np.arange(N) - p + t) % N), 1.0)
        bias = np.where(cnt > 0, np.log(np.maximum(cnt, 1e-300)), -np.inf)
        s = torch.tensor(Q[:, :, b]) @ torch.tensor(K[:, :, b]).T / math.sqrt(d) + torch.tensor(bias)
        out[:, :, b] = (torch.softmax(s, dim=1) @ torch.tensor(V[:, :, b])).numpy()
    return out


@pytest.mark.parametrize("N,d,dv,W", [(30, 12, 6, 7), (64, 32, 32, 16), (20, 8, 8, 29), (100, 16, 8, 1)])
def test_circulant_fa_equals_dpa_and_band_sdpa(N, d, dv, W):
    rng = np.random.default_rng(N + W)
    Q, K, V = rng.standard_normal((N, d, 2)), rng.standard_normal((N, d, 2)), rng.standard_normal((N, dv, 2))
    Of, l, m = O.circulant_fa3(Q, K, V, W, M=64)          # small M: several window blocks
    Od, P = O.circulant_dpa3(Q, K, V, W)
    assert np.allclose(Of, Od, atol=1e-12)
    assert np.allclose(P.sum(axis=0), 1.0)
    assert np.allclose(Of, _torch_band_sdpa(Q, K, V, W), atol=1e-10)
    J = O.circulant_index(N, W)
    S = np.einsum("nkb,wnkb->wnb", Q, K[J]) / math.sqrt(d)
    assert np.allclose(m[:, 0], S.max(axis=0)) and np.allclose(l[:, 0], np.exp(S - S.max(axis=0)).sum(axis=0))


@pytest.mark.parametrize("path", golden_files("circ_"))
def test_golden_circulant_reproduces(path):
    g = load_golden(path)
    W = int(g["W"])
    Oo, l, m = O.circulant_fa3(g["q"], g["k"], g["v"], W)
    assert np.allclose(Oo, g["o"], atol=1e-6)
    assert np.allclose(l, g["l"], rtol=1e-12) and np.allclose(m, g["m"], rtol=1e-12, atol=1e-12)


# --- fused softmax (src/fused_softmax.jl:1-41) ---
@pytest.mark.parametrize("shape,dims", [((7,), 1), ((6, 9), 1), ((6, 9), 2), ((5, 4, 3), 1), ((5, 4, 3), 2)])
def test_fused_softmax_matches_torch(shape, dims):
    rng = np.random.default_rng(sum(shape) + dims)
    S = rng.standard_normal(shape) * 3
    ref = torch.softmax(torch.tensor(S), dim=dims - 1).numpy()
    assert np.allclose(O.fused_softmax(S, dims), ref, atol=1e-14)


def test_fused_softmax_special_values():
    """s .- maximum(s): an all -Inf column is NaN (-Inf - -Inf); -Inf entries
    elsewhere give 0; a +Inf entry makes the vector NaN (Inf - Inf)."""
    S = np.array([[-np.inf, 0.0, 1.0], [-np.inf, -np.inf, np.inf]]).T     # (3, 2) columns
    P = O.fused_softmax(S, 1)
    assert np.isnan(P[:, 1]).all()
    assert P[0, 0] == 0.0 and np.isclose(P[:, 0].sum(), 1.0)


@pytest.mark.parametrize("path", golden_files("softmax_"))
def test_golden_softmax_reproduces(path):
    g = load_golden(path)
    assert np.allclose(O.fused_softmax(g["s"], int(g["dims"])), g["p"], atol=1e-7)
