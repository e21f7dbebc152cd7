"""GPU parity of the reference's remaining exported entry points on this path:
``window`` / ``unwindow`` (src/utils.jl:36-54, NNlib unfold / fold) through
fa_window / fa_unwindow, and the materialising ``dense_dpa`` / ``windowed_dpa``
/ ``block_dpa`` (src/naive/dense.jl:1-35, src/naive/windowed.jl:1-22), checked
against the oracle restatements, the committed golden vectors, and the
reference's own test relation dense_fa ≈ dense_dpa (test/test.jl:19-20)."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from conftest import assert_close, golden_files, load_golden
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


def _bf(rng, shape):
    return torch.tensor(rng.standard_normal(shape)).to(torch.bfloat16).double().numpy()


WGEOMS = [  # (spatial, C, B, ws, stride, pad)
    ((50,), 6, 2, 3, 2, 1),
    ((64,), 4, 1, 7, 7, 3),
    ((13, 11), 5, 2, 3, 2, 1),
    ((16, 16), 8, 1, 4, 4, 0),
    ((20, 18), 3, 2, 7, 7, 3),
    ((9, 7), 2, 1, 5, 1, 2),
    ((6, 5, 4), 3, 2, 3, 2, 1),
]


@pytest.mark.parametrize("dtype", list(DT))
@pytest.mark.parametrize("geom", WGEOMS, ids=lambda g: "x".join(map(str, g[0])) + f"_ws{g[3]}s{g[4]}p{g[5]}")
def test_window_unwindow(fa, geom, dtype):
    sp, C, B, ws, st, pad = geom
    rng = np.random.default_rng(len(sp) * 100 + ws)
    x = _bf(rng, sp + (C, B))
    X = fa.window(fa.jl_tensor(x, DT[dtype]), ws, st, pad)
    torch.cuda.synchronize()
    Xr = O.window(x, ws, st, pad)
    assert tuple(X.shape) == Xr.shape
    assert np.array_equal(_np(X), Xr), "window is exact data movement"
    Y = _bf(rng, Xr.shape)
    y = fa.unwindow(fa.jl_tensor(Y, DT[dtype]), sp + (C, B), ws, st, pad)
    torch.cuda.synchronize()
    yr = O.unwindow(Y, sp + (C, B), ws, st, pad)
    if st >= ws:   # no overlap: a pure scatter, exact
        assert np.array_equal(_np(y), yr)
    else:          # sums of overlapping windows, accumulated in fp32, rounded once
        assert_close(_np(y), yr, dtype, "unwindow")


@pytest.mark.parametrize("dtype", list(DT))
@pytest.mark.parametrize("path", golden_files("dense_"), ids=lambda p: p.split("/")[-1][:-4])
def test_dense_dpa_golden(fa, path, dtype):
    g = load_golden(path)
    q, k, v = (fa.jl_tensor(g[x], DT[dtype]) for x in ("q", "k", "v"))
    y, P = fa.dense_dpa(q, k, v)
    torch.cuda.synchronize()
    assert_close(_np(y), g["y"], dtype, "y")
    if P.numel() <= 4_000_000:
        _, Pr = O.dense_dpa(g["q"], g["k"], g["v"])
        assert tuple(P.shape) == Pr.shape
        assert_close(_np(P), Pr, dtype, "P")
        assert np.allclose(_np(P).sum(axis=1), 1.0, atol=2e-2 if dtype != "float32" else 1e-5)


@pytest.mark.parametrize("dtype", list(DT))
def test_dense_fa_matches_dense_dpa(fa, dtype):
    """test/test.jl:19: dense_fa(q, k, v)[1] ≈ dense_dpa(q, k, v)[1], with the test's own shape."""
    rng = np.random.default_rng(11)
    q, k = _bf(rng, (30, 12, 2)), _bf(rng, (30, 12, 2))
    v = _bf(rng, (30, 6, 2))
    Q, K, V = (fa.jl_tensor(a, DT[dtype]) for a in (q, k, v))
    y1 = _np(fa.dense_fa(Q, K, V)[0])
    y2 = _np(fa.dense_dpa(Q, K, V)[0])
    assert_close(y1, y2, dtype, "dense_fa vs dense_dpa")


@pytest.mark.parametrize("dtype", list(DT))
@pytest.mark.parametrize("path", golden_files("wind_") + golden_files("block_"),
                         ids=lambda p: p.split("/")[-1][:-4])
def test_windowed_dpa_golden(fa, path, dtype):
    g = load_golden(path)
    ws, st, pad = int(g["ws"]), int(g["stride"]), int(g["pad"])
    q, k, v = (fa.jl_tensor(g[x], DT[dtype]) for x in ("q", "k", "v"))
    y, P = fa.windowed_dpa(q, k, v, ws, st, pad)
    torch.cuda.synchronize()
    assert_close(_np(y), g["y"], dtype, "y", nan_ok=True)
    T = ws ** (q.dim() - 2)
    assert P.shape[0] == T and P.shape[1] == T and P.shape[3] == q.shape[-1]
    yf = _np(fa.windowed_fa(q, k, v, ws, stride=st, pad=pad)[0])
    assert_close(_np(y), yf, dtype, "windowed_dpa vs windowed_fa", nan_ok=True)


def test_block_dpa_is_windowed_dpa_default(fa):
    rng = np.random.default_rng(5)
    x = fa.jl_tensor(_bf(rng, (12, 12, 8, 2)), torch.float32)
    a = fa.block_dpa(x, x, x, 3)
    b = fa.windowed_dpa(x, x, x, 3)
    torch.cuda.synchronize()
    for u, w in zip(a, b):
        assert torch.equal(torch.nan_to_num(u, 7.0), torch.nan_to_num(w, 7.0))
