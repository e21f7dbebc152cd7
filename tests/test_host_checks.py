"""CPU tests of the Python mirror's argument validation (fa_hip): every shape /
dtype problem must raise DimensionMismatch BEFORE any pointer reaches the C ABI
(a wrong l / m dtype or a mis-shaped gradient input would otherwise make the
kernels read or write out of bounds).  No device is touched."""
from __future__ import annotations

import pytest
import torch

import fa_hip
from fa_hip import DimensionMismatch


def jl(shape, dtype=torch.bfloat16):
    return fa_hip.jl_empty(shape, dtype, device="cpu")


def test_dense_backward_rejects_non_f32_stats():
    N, d, B = 16, 8, 2
    Q, K, V, O, dO = (jl((N, d, B)) for _ in range(5))
    for bad in (torch.bfloat16, torch.float16, torch.float64):
        with pytest.raises(DimensionMismatch, match="float32"):
            fa_hip.dense_fa_backward(Q, K, V, O, dO, jl((N, 1, B), bad), jl((N, 1, B), torch.float32))
        with pytest.raises(DimensionMismatch, match="float32"):
            fa_hip.dense_fa_backward(Q, K, V, O, dO, jl((N, 1, B), torch.float32), jl((N, 1, B), bad))


def test_dense_backward_rejects_bad_shapes():
    N, d, B = 16, 8, 2
    Q, K, V = jl((N, d, B)), jl((N, d, B)), jl((N, d, B))
    f = lambda s: jl(s, torch.float32)
    with pytest.raises(DimensionMismatch):
        fa_hip.dense_fa_backward(Q, K, V, jl((N, d + 1, B)), jl((N, d, B)), f((N, 1, B)), f((N, 1, B)))
    with pytest.raises(DimensionMismatch):
        fa_hip.dense_fa_backward(Q, K, V, jl((N, d, B)), jl((N, d, B)), f((N - 1, 1, B)), f((N, 1, B)))


def _win_inputs(S=(14, 14), d=8, dv=8, B=2, ws=7, dtype=torch.bfloat16):
    q, k = jl(S + (d, B), dtype), jl(S + (d, B), dtype)
    v, y, dy = jl(S + (dv, B), dtype), jl(S + (dv, B), dtype), jl(S + (dv, B), dtype)
    L = 1
    for s in S:
        L *= (s + 2 * ((ws - 1) // 2) - ws) // ws + 1
    T = ws ** len(S)
    return q, k, v, y, dy, jl((T, 1, L, B), torch.float32), jl((T, 1, L, B), torch.float32)


def test_windowed_backward_rejects_bad_shapes():
    q, k, v, y, dy, l, m = _win_inputs()
    S = tuple(q.shape[:2])
    bad = {
        "k": jl((S[0], S[1] - 1, 8, 2)),
        "y": jl(S + (8 + 1, 2)),
        "dy": jl((S[0] + 1, S[1], 8, 2)),
        "l": jl((49, 1, 3, 2), torch.float32),
        "m": jl((48, 1, 4, 2), torch.float32),
    }
    args = dict(q=q, k=k, v=v, y=y, dy=dy, l=l, m=m)
    for name, t in bad.items():
        a = dict(args)
        a[name] = t
        with pytest.raises(DimensionMismatch):
            fa_hip.windowed_fa_backward(a["q"], a["k"], a["v"], a["y"], a["dy"], a["l"], a["m"], 7)


def test_windowed_backward_rejects_non_f32_stats():
    q, k, v, y, dy, l, m = _win_inputs()
    lb = jl(tuple(l.shape), torch.bfloat16)
    with pytest.raises(DimensionMismatch, match="float32"):
        fa_hip.windowed_fa_backward(q, k, v, y, dy, lb, m, 7)


def test_valid_windowed_backward_shapes_reach_the_device_check():
    """A well-formed call gets past every shape check and stops only at the
    device check (CPU tensors): the checks do not reject valid geometry."""
    q, k, v, y, dy, l, m = _win_inputs()
    with pytest.raises(TypeError, match="ROCm device"):
        fa_hip.windowed_fa_backward(q, k, v, y, dy, l, m, 7)


def test_circulant_band_index_matches_oracle():
    """fa_hip.circulant_band_index (vectorised, used by circulant_dpa) equals the
    oracle's loop over the reference's cartesian_circulant (src/utils.jl:6-17),
    including even W, W = 1 and W > N."""
    import numpy as np
    from oracle import fa_oracle as O
    for N, W in [(10, 3), (17, 5), (9, 4), (8, 11), (30, 1), (64, 65), (5, 5), (100, 16)]:
        J = fa_hip.circulant_band_index(N, W, "cpu").numpy()
        assert np.array_equal(J, O.circulant_index(N, W)), (N, W)
