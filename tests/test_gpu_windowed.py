"""GPU parity tests: windowed / block attention through the C ABI
(fa_windowed_fwd / fa_windowed_bwd) vs the oracle restatement of
windowed_fa (src/windowed.jl:3-23) with NNlib unfold/fold geometry pinned to
torch F.unfold/F.fold (tests/test_oracle.py), on the committed golden vectors
(1-D, 2-D, 3-D; stride = ws and stride < ws; default and zero pad; the NaN
tail of Appendix A.7) and BASELINE configs[2]."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from conftest import assert_close, assert_lm_close, golden_files, load_golden
from oracle import fa_oracle as O

pytestmark = pytest.mark.gpu
DT = {"float32": torch.float32, "bfloat16": torch.bfloat16, "float16": torch.float16}
GTOL = {"float32": 2e-5, "bfloat16": 2e-2, "float16": 5e-3}


@pytest.fixture(scope="module")
def fa():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm device")
    import fa_hip
    fa_hip.lib()
    return fa_hip


def _np(t):
    return t.detach().float().cpu().numpy().astype(np.float64)


@pytest.mark.parametrize("dtype", list(DT))
@pytest.mark.parametrize("path", golden_files("wind_") + golden_files("block_"),
                         ids=lambda p: p.split("/")[-1][:-4])
def test_windowed_golden(fa, path, dtype):
    g = load_golden(path)
    ws, st, pad = int(g["ws"]), int(g["stride"]), int(g["pad"])
    q, k, v = (fa.jl_tensor(g[x], DT[dtype]) for x in ("q", "k", "v"))
    y, l, m = fa.windowed_fa(q, k, v, ws, stride=st, pad=pad)
    torch.cuda.synchronize()
    assert tuple(y.shape) == g["y"].shape and tuple(l.shape) == g["l"].shape
    assert_close(_np(y), g["y"], dtype, "y", nan_ok=True)
    assert_lm_close(_np(l), g["l"], dtype, "l")
    assert_lm_close(_np(m), g["m"], dtype, "m")


@pytest.mark.parametrize("dtype", list(DT))
@pytest.mark.parametrize("path", golden_files("wind_") + golden_files("block_"),
                         ids=lambda p: p.split("/")[-1][:-4])
def test_windowed_backward_golden(fa, path, dtype):
    g = load_golden(path)
    ws, st, pad = int(g["ws"]), int(g["stride"]), int(g["pad"])
    q, k, v, dy = (fa.jl_tensor(g[x], DT[dtype]) for x in ("q", "k", "v", "dy"))
    y, l, m = fa.windowed_fa(q, k, v, ws, stride=st, pad=pad)
    dq, dk, dv = fa.windowed_fa_backward(q, k, v, y, dy, l, m, ws, stride=st, pad=pad)
    torch.cuda.synchronize()
    for a, b, nm in ((dq, g["dq"], "dq"), (dk, g["dk"], "dk"), (dv, g["dv"], "dv")):
        x = _np(a)
        scale = max(np.abs(b).max(), 1e-2)
        err = np.abs(x - b).max() / scale
        assert np.all(np.isfinite(x)) and err <= GTOL[dtype], f"{nm}: {err:.2e}"


def test_block_fa_is_windowed_with_stride_ws(fa):
    rng = np.random.default_rng(4)
    x = fa.jl_tensor(rng.standard_normal((16, 12, 8, 2)), torch.float32)
    a = fa.block_fa(x, x, x, 4)
    b = fa.windowed_fa(x, x, x, 4, stride=4, pad=0)
    torch.cuda.synchronize()
    for u, w in zip(a, b):
        assert torch.equal(u, w)


def test_config3_full_size(fa):
    """BASELINE configs[2]: 2-D 128x128 tokens, ws=7 (stride 7, pad 3 → 19x19 = 361
    windows of 49 tokens), d = 64, bf16, B = 2; oracle on the full image."""
    rng = np.random.default_rng(7)
    bf = lambda a: torch.tensor(a).to(torch.bfloat16).double().numpy()
    q, k, v = (bf(rng.standard_normal((128, 128, 64, 2))) for _ in range(3))
    y, l, m = fa.windowed_fa(*(fa.jl_tensor(a, torch.bfloat16) for a in (q, k, v)), 7)
    torch.cuda.synchronize()
    yr, lr, mr = O.windowed_fa(q, k, v, 7, 7, 3)
    assert l.shape == (49, 1, 361, 2)
    assert_close(_np(y), yr, "bfloat16", "y", nan_ok=True)
    assert_lm_close(_np(l), lr, "bfloat16", "l")
    assert_lm_close(_np(m), mr, "bfloat16", "m")


@pytest.mark.parametrize("B,mode", [(1, 0), (1, 3), (3, 13)])
def test_config2_backward_full_size_window_pairing(fa, B, mode):
    """BASELINE configs[2] backward on the full image against the oracle's chain rule,
    through the per-window kernel with two windows per workgroup (auto at B = 1: 361
    windows; forced at B = 3, where a pair straddles two images since 361 is odd) and
    with one (mode 3); the two layouts give the same bits."""
    rng = np.random.default_rng(17 + B)
    bf = lambda a: torch.tensor(a).to(torch.bfloat16).double().numpy()
    q, k, v, dy = (bf(rng.standard_normal((128, 128, 64, B))) for _ in range(4))
    Q, K, V, DY = (fa.jl_tensor(a, torch.bfloat16) for a in (q, k, v, dy))
    y, l, m = fa.windowed_fa(Q, K, V, 7)
    L = fa.lib()
    grads = {}
    for md in (mode, 3):
        old = L.fa_debug_set_win_composed(md)
        try:
            grads[md] = [t.clone() for t in fa.windowed_fa_backward(Q, K, V, y, DY, l, m, 7)]
            torch.cuda.synchronize()
        finally:
            L.fa_debug_set_win_composed(old)
    for a, b_ in zip(grads[mode], grads[3]):
        assert torch.equal(a, b_), "window pairing changed the bits"
    ref = O.windowed_fa_backward(q, k, v, dy, 7, 7, 3)
    for a, b_, nm in zip(grads[mode], ref, ("dq", "dk", "dv")):
        assert_close(_np(a), b_, "bfloat16", nm)
