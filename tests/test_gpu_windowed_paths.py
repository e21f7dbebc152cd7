"""GPU parity of every fused windowed-forward kernel, each forced in turn
(fa_debug_set_win_composed: 1 composed gather→dense→fold, 2 register-gather,
3 one-window row-shift (ws <= 7) / row-scatter (ws = 8), 4 four-window
row-staged, 5 one-window row-scatter, 6 two-window row-shift, 12 three-window row-shift, 10 the eight-window strip kernel
with rotated slots and analytic padding columns), against the oracle restatement of
windowed_fa (src/windowed.jl:3-23, NNlib unfold/fold geometry) on geometries
chosen for the row-staged kernels' edge handling: windows hanging over the
left / right / bottom image edge, odd and even window x-starts (the row-shift
kernel's dword-aligned 16-B loads), pad >= ws, stride > ws (uncovered pixels
are NaN), ws = 8, and head dims below / between the compiled classes."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from conftest import assert_close, assert_lm_close
from oracle import fa_oracle as O

pytestmark = pytest.mark.gpu

GEOMS = [  # (W, H, ws, stride, pad)
    (16, 16, 3, 3, 1),
    (24, 13, 5, 5, 2),
    (32, 20, 7, 7, 3),
    (16, 9, 7, 9, 0),
    (8, 8, 7, 7, 6),
    (40, 24, 6, 6, 2),
    (24, 16, 8, 8, 3),
    (48, 17, 7, 8, 1),
]
DIMS = [(64, 64), (32, 64), (64, 32), (20, 48)]


@pytest.fixture(scope="module")
def fa():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm device")
    import fa_hip
    fa_hip.lib()
    return fa_hip


def _np(t):
    return t.detach().float().cpu().numpy().astype(np.float64)


@pytest.mark.parametrize("path", [0, 1, 2, 3, 4, 5, 6, 10, 12])
@pytest.mark.parametrize("geom", GEOMS, ids=lambda g: "W{}H{}ws{}s{}p{}".format(*g))
def test_windowed_forced_path(fa, geom, path):
    W, H, ws, st, pad = geom
    rng = np.random.default_rng(W * 1000 + H * 10 + ws)
    bf = lambda a: torch.tensor(a).to(torch.bfloat16).double().numpy()
    L = fa.lib()
    old = L.fa_debug_set_win_composed(path)
    try:
        for (d, dv) in DIMS:
            B = 2
            q, k = (bf(rng.standard_normal((W, H, d, B))) for _ in range(2))
            v = bf(rng.standard_normal((W, H, dv, B)))
            y, l, m = fa.windowed_fa(*(fa.jl_tensor(a, torch.bfloat16) for a in (q, k, v)), ws,
                                     stride=st, pad=pad)
            torch.cuda.synchronize()
            yr, lr, mr = O.windowed_fa(q, k, v, ws, st, pad)
            tag = f"path {path} d {d} dv {dv}"
            assert_close(_np(y), yr, "bfloat16", f"y ({tag})", nan_ok=True)
            assert_lm_close(_np(l), lr, "bfloat16", f"l ({tag})")
            assert_lm_close(_np(m), mr, "bfloat16", f"m ({tag})")
    finally:
        L.fa_debug_set_win_composed(old)


DIMS128 = [(128, 128), (96, 64), (64, 128), (128, 40)]


@pytest.mark.parametrize("path", [0, 1])
@pytest.mark.parametrize("geom", GEOMS, ids=lambda g: "W{}H{}ws{}s{}p{}".format(*g))
def test_windowed_wide_heads(fa, geom, path):
    """d or dv in (64, 128]: path 0 runs the one-window row-shift kernel at 128
    features where the geometry allows (stride >= ws, ws <= 7), the composed
    path otherwise; path 1 forces the composed path.  Same oracle."""
    W, H, ws, st, pad = geom
    rng = np.random.default_rng(W * 977 + H * 13 + ws)
    bf = lambda a: torch.tensor(a).to(torch.bfloat16).double().numpy()
    L = fa.lib()
    old = L.fa_debug_set_win_composed(path)
    try:
        for (d, dv) in DIMS128:
            B = 2
            q, k = (bf(rng.standard_normal((W, H, d, B))) for _ in range(2))
            v = bf(rng.standard_normal((W, H, dv, B)))
            y, l, m = fa.windowed_fa(*(fa.jl_tensor(a, torch.bfloat16) for a in (q, k, v)), ws,
                                     stride=st, pad=pad)
            torch.cuda.synchronize()
            yr, lr, mr = O.windowed_fa(q, k, v, ws, st, pad)
            tag = f"path {path} d {d} dv {dv}"
            assert_close(_np(y), yr, "bfloat16", f"y ({tag})", nan_ok=True)
            assert_lm_close(_np(l), lr, "bfloat16", f"l ({tag})")
            assert_lm_close(_np(m), mr, "bfloat16", f"m ({tag})")
    finally:
        L.fa_debug_set_win_composed(old)


BWD_GEOMS = [g for g in GEOMS if g[3] >= g[2] and g[2] <= 7]   # stride >= ws, ws <= 7: the fused backward


@pytest.mark.parametrize("path", [0, 1])
@pytest.mark.parametrize("geom", BWD_GEOMS, ids=lambda g: "W{}H{}ws{}s{}p{}".format(*g))
def test_windowed_backward_paths(fa, geom, path):
    """Fused windowed backward (path 0: win_bwd_rows, 64- or 128-feature class) and the composed
    gather → dense backward → fold path (1) vs the oracle chain rule."""
    W, H, ws, st, pad = geom
    rng = np.random.default_rng(W * 7 + H * 3 + ws)
    bf = lambda a: torch.tensor(a).to(torch.bfloat16).double().numpy()
    L = fa.lib()
    old = L.fa_debug_set_win_composed(path)
    try:
        for (d, dv) in DIMS + DIMS128:   # d, dv > 64: the fused kernel at 128 features
            B = 2
            q, k = (bf(rng.standard_normal((W, H, d, B))) for _ in range(2))
            v, dy = (bf(rng.standard_normal((W, H, dv, B))) for _ in range(2))
            Q, K, V, DY = (fa.jl_tensor(a, torch.bfloat16) for a in (q, k, v, dy))
            y, l, m = fa.windowed_fa(Q, K, V, ws, stride=st, pad=pad)
            dq, dk, dvv = fa.windowed_fa_backward(Q, K, V, y, DY, l, m, ws, stride=st, pad=pad)
            torch.cuda.synchronize()
            ref = O.windowed_fa_backward(q, k, v, dy, ws, st, pad)
            for a, b_, nm in zip((dq, dk, dvv), ref, ("dq", "dk", "dv")):
                x = _np(a)
                scale = max(np.abs(b_).max(), 1e-2)
                err = np.abs(x - b_).max() / scale
                assert np.all(np.isfinite(x)) and err <= 2e-2, f"path {path} d {d} dv {dv} {nm}: {err:.2e}"
    finally:
        L.fa_debug_set_win_composed(old)


@pytest.mark.parametrize("path", [0, 1])
@pytest.mark.parametrize("geom", GEOMS, ids=lambda g: "W{}H{}ws{}s{}p{}".format(*g))
def test_windowed_f32_paths(fa, geom, path):
    """fp32: the fused exact-f32 MFMA windowed kernel (path 0, stride >= ws) and
    the composed path (1) against the float64 oracle at the fp32 tolerance."""
    W, H, ws, st, pad = geom
    rng = np.random.default_rng(W * 11 + H + ws)
    L = fa.lib()
    old = L.fa_debug_set_win_composed(path)
    try:
        for (d, dv) in DIMS:
            B = 2
            q, k = (rng.standard_normal((W, H, d, B)) for _ in range(2))
            v = rng.standard_normal((W, H, dv, B))
            y, l, m = fa.windowed_fa(*(fa.jl_tensor(a, torch.float32) for a in (q, k, v)), ws, stride=st, pad=pad)
            torch.cuda.synchronize()
            yr, lr, mr = O.windowed_fa(q, k, v, ws, st, pad)
            tag = f"path {path} d {d} dv {dv}"
            assert_close(_np(y), yr, "float32", f"y ({tag})", nan_ok=True)
            assert_lm_close(_np(l), lr, "float32", f"l ({tag})")
            assert_lm_close(_np(m), mr, "float32", f"m ({tag})")
    finally:
        L.fa_debug_set_win_composed(old)


@pytest.mark.parametrize("path", [0, 1])
@pytest.mark.parametrize("geom", [g for g in GEOMS if g[3] >= g[2]], ids=lambda g: "W{}H{}ws{}s{}p{}".format(*g))
def test_windowed_backward_f32_paths(fa, geom, path):
    """fp32 windowed backward: the fused exact-f32 MFMA kernel (path 0) and the
    composed path (1) against the float64 oracle chain rule (fp32 tolerance)."""
    W, H, ws, st, pad = geom
    rng = np.random.default_rng(W * 13 + H + ws)
    L = fa.lib()
    old = L.fa_debug_set_win_composed(path)
    try:
        for (d, dv) in DIMS:
            B = 2
            q, k = (rng.standard_normal((W, H, d, B)) for _ in range(2))
            v, dy = (rng.standard_normal((W, H, dv, B)) for _ in range(2))
            Q, K, V, DY = (fa.jl_tensor(a, torch.float32) for a in (q, k, v, dy))
            y, l, m = fa.windowed_fa(Q, K, V, ws, stride=st, pad=pad)
            dq, dk, dvv = fa.windowed_fa_backward(Q, K, V, y, DY, l, m, ws, stride=st, pad=pad)
            torch.cuda.synchronize()
            ref = O.windowed_fa_backward(q, k, v, dy, ws, st, pad)
            for a, b_, nm in zip((dq, dk, dvv), ref, ("dq", "dk", "dv")):
                x = _np(a)
                scale = max(np.abs(b_).max(), 1e-2)
                err = np.abs(x - b_).max() / scale
                assert np.all(np.isfinite(x)) and err <= 2e-5, f"path {path} d {d} dv {dv} {nm}: {err:.2e}"
    finally:
        L.fa_debug_set_win_composed(old)


@pytest.mark.parametrize("path", [0, 3, 6, 10, 12])
def test_windowed_nonfinite_stays_in_its_window(fa, path):
    """An inf in one pixel's k and v reaches only the window holding that pixel, as in
    the reference, where windows are disjoint token sets.  The fused kernels load 8-pixel
    rows that also hold a neighbour window's pixel (pixel 10 sits in the row load of
    the window starting at 11); those slots must be masked (row-shift kernels: zeroed
    in staging; LDS-DMA kernels: keys selected to -inf, V fragments ANDed with the slot
    mask)."""
    W, H, ws, st, pad = 32, 20, 7, 7, 3
    rng = np.random.default_rng(5)
    bf = lambda a: torch.tensor(a).to(torch.bfloat16).double().numpy()
    d = dv = 64
    q, k, v = (bf(rng.standard_normal((W, H, d, 1))) for _ in range(3))
    k[10, 10, 5, 0] = np.inf
    v[10, 10, 3, 0] = np.inf
    L = fa.lib()
    old = L.fa_debug_set_win_composed(path)
    try:
        y, l, m = fa.windowed_fa(*(fa.jl_tensor(a, torch.bfloat16) for a in (q, k, v)), ws, stride=st, pad=pad)
        torch.cuda.synchronize()
    finally:
        L.fa_debug_set_win_composed(old)
    with np.errstate(invalid="ignore", over="ignore"):
        yr, lr, mr = O.windowed_fa(q, k, v, ws, st, pad)
    O0 = (W + 2 * pad - ws) // st + 1
    inwin = np.zeros((W, H), bool)
    inwin[4:11, 4:11] = True                      # window (1, 1): x, y in [4, 11)
    # rows 18, 19 are covered by no window: NaN there in both (0/0, as the reference)
    yo, yro = _np(y)[~inwin], yr[~inwin]
    assert not np.isinf(yo).any(), f"path {path}: inf outside the window holding the inf"
    assert_close(yo, yro, "bfloat16", f"y outside the window (path {path})", nan_ok=True)
    keep = np.ones(lr.shape[2], bool)
    keep[1 + O0 * 1] = False
    assert_lm_close(_np(l)[:, :, keep], lr[:, :, keep], "bfloat16", f"l (path {path})")
    assert_lm_close(_np(m)[:, :, keep], mr[:, :, keep], "bfloat16", f"m (path {path})")


STRIP_GEOMS = [  # stride == ws, width % 8 == 0 (the strip kernel's eligibility)
    (32, 20, 7, 7, 3),      # 6 windows: one partial strip
    (128, 16, 7, 7, 3),     # configs[2]'s width: 19 windows = 8 + 8 + 3
    (120, 9, 7, 7, 0),      # 17 windows, the last pixels uncovered (NaN)
    (64, 13, 6, 6, 2),
    (72, 12, 5, 5, 2),
    (64, 17, 3, 3, 1),
    (16, 8, 7, 7, 6),       # pad close to ws: windows hang over both edges
    (112, 10, 7, 7, 5),
    (64, 12, 4, 4, 1),      # even ws, odd pad: no first-strip width aligns the strip ends (2-B end stores)
    (48, 10, 6, 6, 1),
    (200, 9, 7, 7, 3),      # 29 windows: first strip 5 (ends on 16-B chunks), then 8 + 8 + 8
]


@pytest.mark.parametrize("dtype", ["bfloat16", "float16"])
@pytest.mark.parametrize("geom", STRIP_GEOMS, ids=lambda g: "W{}H{}ws{}s{}p{}".format(*g))
def test_windowed_strip_kernel(fa, geom, dtype):
    """Mode 10 (win_strip: eight adjacent windows per workgroup, channel-streamed LDS-DMA,
    y stored as 16-B chunks of the strip) vs the oracle, and against the two-window
    row-shift kernel (mode 6) within one bf16/f16 rounding of y (its fused
    O·(1/l) rounding differs in the last bit)."""
    W, H, ws, st, pad = geom
    tdt = torch.bfloat16 if dtype == "bfloat16" else torch.float16
    rng = np.random.default_rng(W * 37 + H * 11 + ws)
    cast = lambda a: torch.tensor(a).to(tdt).double().numpy()
    L = fa.lib()
    for (d, dv) in DIMS:
        B = 3
        q, k = (cast(rng.standard_normal((W, H, d, B))) for _ in range(2))
        v = cast(rng.standard_normal((W, H, dv, B)))
        outs = {}
        for path in (10, 6):
            old = L.fa_debug_set_win_composed(path)
            try:
                outs[path] = fa.windowed_fa(*(fa.jl_tensor(a, tdt) for a in (q, k, v)), ws, stride=st, pad=pad)
                torch.cuda.synchronize()
            finally:
                L.fa_debug_set_win_composed(old)
        y, l, m = outs[10]
        yr, lr, mr = O.windowed_fa(q, k, v, ws, st, pad)
        tag = f"d {d} dv {dv}"
        assert_close(_np(y), yr, dtype, f"y ({tag})", nan_ok=True)
        assert_lm_close(_np(l), lr, dtype, f"l ({tag})")
        assert_lm_close(_np(m), mr, dtype, f"m ({tag})")
        y6, l6, m6 = outs[6]
        assert_close(_np(y), _np(y6), dtype, f"y vs mode 6 ({tag})", nan_ok=True)
        assert_lm_close(_np(l), _np(l6), dtype, f"l vs mode 6 ({tag})")
        assert_lm_close(_np(m), _np(m6), dtype, f"m vs mode 6 ({tag})")


def test_windowed_strip_full_size(fa):
    """configs[2] at B = 32 runs the strip kernel by default (>= kStripMin strips): the
    oracle on two images, and the rows / pixels no other path wrote are all set."""
    W = H = 128
    B, d = 32, 64
    g = torch.Generator(device="cuda").manual_seed(9)
    q, k, v = (fa.jl_tensor(torch.randn((W, H, d, B), generator=g, device="cuda"), torch.bfloat16) for _ in range(3))
    y, l, m = fa.windowed_fa(q, k, v, 7)
    torch.cuda.synchronize()
    assert torch.isfinite(y.float()).all()
    for b in (0, 31):
        sl = lambda t: _np(t[..., b:b + 1])
        yr, lr, mr = O.windowed_fa(sl(q), sl(k), sl(v), 7, 7, 3)
        assert_close(sl(y), yr, "bfloat16", f"y image {b}")
        assert_lm_close(_np(l[:, :, :, b:b + 1]), lr, "bfloat16", f"l image {b}")
        assert_lm_close(_np(m[:, :, :, b:b + 1]), mr, "bfloat16", f"m image {b}")


def _bwd_grads(fa, q, k, v, dy, ws, st, pad, dt, path):
    L = fa.lib()
    old = L.fa_debug_set_win_composed(path)
    try:
        Q, K, V, DY = (fa.jl_tensor(a, dt) for a in (q, k, v, dy))
        y, l, m = fa.windowed_fa(Q, K, V, ws, stride=st, pad=pad)
        g = fa.windowed_fa_backward(Q, K, V, y, DY, l, m, ws, stride=st, pad=pad)
        torch.cuda.synchronize()
        return g
    finally:
        L.fa_debug_set_win_composed(old)


@pytest.mark.parametrize("dtype", ["bfloat16", "float16"])
@pytest.mark.parametrize("geom", STRIP_GEOMS, ids=lambda g: "W{}H{}ws{}s{}p{}".format(*g))
def test_windowed_backward_strip_kernel(fa, geom, dtype):
    """Mode 10 backward (win_bwd_strip: eight windows per workgroup, D = rowsum(P ∘ dP),
    identity-MFMA transposes, 16-B gradient chunk stores) vs the oracle chain rule, and
    close to the one-window kernel (mode 3, win_bwd_rows, D from y)."""
    W, H, ws, st, pad = geom
    tdt = torch.bfloat16 if dtype == "bfloat16" else torch.float16
    rng = np.random.default_rng(W * 41 + H * 5 + ws)
    cast = lambda a: torch.tensor(a).to(tdt).double().numpy()
    for (d, dv) in DIMS:
        B = 3
        q, k = (cast(rng.standard_normal((W, H, d, B))) for _ in range(2))
        v, dy = (cast(rng.standard_normal((W, H, dv, B))) for _ in range(2))
        g10 = _bwd_grads(fa, q, k, v, dy, ws, st, pad, tdt, 10)
        g3 = _bwd_grads(fa, q, k, v, dy, ws, st, pad, tdt, 3)
        ref = O.windowed_fa_backward(q, k, v, dy, ws, st, pad)
        for a, a3, b_, nm in zip(g10, g3, ref, ("dq", "dk", "dv")):
            x, x3 = _np(a), _np(a3)
            scale = max(np.abs(b_).max(), 1e-2)
            err = np.abs(x - b_).max() / scale
            assert np.all(np.isfinite(x)) and err <= 2e-2, f"d {d} dv {dv} {nm}: {err:.2e} vs the oracle"
            err3 = np.abs(x - x3).max() / scale
            assert err3 <= 2e-2, f"d {d} dv {dv} {nm}: {err3:.2e} vs mode 3"


@pytest.mark.parametrize("path", [3, 10])
def test_windowed_backward_nonfinite_stays_in_its_window(fa, path):
    """An inf in one pixel's q, k, v and dy changes the gradients of that pixel's window
    only: every other pixel's dq, dk, dv is bitwise the inf-free result (the neighbour
    window's 8-pixel row loads hold the pixel, masked by selects)."""
    W, H, ws, st, pad = 32, 20, 7, 7, 3
    rng = np.random.default_rng(6)
    bf = lambda a: torch.tensor(a).to(torch.bfloat16).double().numpy()
    d = dv = 64
    q, k, v, dy = (bf(rng.standard_normal((W, H, d, 1))) for _ in range(4))
    clean = _bwd_grads(fa, q, k, v, dy, ws, st, pad, torch.bfloat16, path)
    for a in (q, k, v, dy):
        a[10, 10, 5, 0] = np.inf
    dirty = _bwd_grads(fa, q, k, v, dy, ws, st, pad, torch.bfloat16, path)
    inwin = torch.zeros((W, H), dtype=torch.bool, device="cuda")
    inwin[4:11, 4:11] = True
    for c, g, nm in zip(clean, dirty, ("dq", "dk", "dv")):
        out = ~inwin
        assert torch.equal(c[out].view(torch.int16), g[out].view(torch.int16)), f"path {path} {nm} changed outside"


def test_windowed_backward_strip_full_size(fa):
    """configs[2] at B = 32 runs the strip backward by default: the oracle on two images."""
    W = H = 128
    B, d = 32, 64
    g = torch.Generator(device="cuda").manual_seed(10)
    q, k, v, dy = (fa.jl_tensor(torch.randn((W, H, d, B), generator=g, device="cuda"), torch.bfloat16)
                   for _ in range(4))
    y, l, m = fa.windowed_fa(q, k, v, 7)
    dq, dk, dvv = fa.windowed_fa_backward(q, k, v, y, dy, l, m, 7)
    torch.cuda.synchronize()
    for b in (0, 31):
        sl = lambda t: _np(t[..., b:b + 1])
        ref = O.windowed_fa_backward(sl(q), sl(k), sl(v), sl(dy), 7, 7, 3)
        for a, b_, nm in zip((dq, dk, dvv), ref, ("dq", "dk", "dv")):
            x = sl(a)
            err = np.abs(x - b_).max() / max(np.abs(b_).max(), 1e-2)
            assert np.all(np.isfinite(x)) and err <= 2e-2, f"image {b} {nm}: {err:.2e}"


@pytest.mark.parametrize("B", [9, 40])
def test_windowed_backward_strip_dynamic_deal_every_image(fa, B):
    """The strip backward's dynamic deal (one workgroup per CU; strips b, b + G, then a
    counter in the workspace) at strip counts that are not a multiple of the grid:
    B = 9 (513 strips: 256 static first strips, 256 second, one drawn) and B = 40 (2280
    strips: 1768 drawn, a ragged last round).  Every image of the default path's
    gradients must match the one-window kernel (mode 3) within the 16-bit tolerance
    (a strip the deal skipped would keep whatever the fresh output buffer held).  Run
    twice: which workgroup draws which strip changes from run to run, the gradients
    must not (bitwise)."""
    W = H = 128
    d = 64
    g = torch.Generator(device="cuda").manual_seed(11 + B)
    q, k, v, dy = (fa.jl_tensor(torch.randn((W, H, d, B), generator=g, device="cuda"), torch.bfloat16)
                   for _ in range(4))
    y, l, m = fa.windowed_fa(q, k, v, 7)
    runs = [[t.clone() for t in fa.windowed_fa_backward(q, k, v, y, dy, l, m, 7)] for _ in range(2)]
    torch.cuda.synchronize()
    L = fa.lib()
    old = L.fa_debug_set_win_composed(3)
    try:
        ref = fa.windowed_fa_backward(q, k, v, y, dy, l, m, 7)
        torch.cuda.synchronize()
    finally:
        L.fa_debug_set_win_composed(old)
    for a, a2, r, nm in zip(runs[0], runs[1], ref, ("dq", "dk", "dv")):
        assert torch.equal(a, a2), f"{nm}: two runs of the dynamic deal differ"
        x, xr = a.float(), r.float()
        assert torch.isfinite(x).all(), f"{nm}: non-finite gradient (a strip not computed?)"
        per_image = ((x - xr).abs().amax(dim=(0, 1, 2)) / xr.abs().amax(dim=(0, 1, 2)).clamp_min(1e-2))
        assert float(per_image.max()) <= 2e-2, f"{nm}: worst image {int(per_image.argmax())} err {float(per_image.max()):.2e}"


@pytest.mark.parametrize("grid", [37, 200, 257])
def test_windowed_backward_strip_deal_any_grid(fa, grid):
    """The strip backward's XCD-group deal at grid sizes other than one workgroup per CU
    (fa_debug_set_win_bwd_grid: 37 leaves groups of 4 and 5 workgroups, 200 an uneven
    split over the 8 groups, 257 is capped at the strip count's grid rule only): every
    strip is computed exactly once, so the gradients are bitwise those of the default grid."""
    import ctypes
    W = H = 128
    B, d = 8, 64
    g = torch.Generator(device="cuda").manual_seed(90 + grid)
    q, k, v, dy = (fa.jl_tensor(torch.randn((W, H, d, B), generator=g, device="cuda"), torch.bfloat16)
                   for _ in range(4))
    y, l, m = fa.windowed_fa(q, k, v, 7)
    ref = [t.clone() for t in fa.windowed_fa_backward(q, k, v, y, dy, l, m, 7)]
    L = fa.lib()
    L.fa_debug_set_win_bwd_grid.argtypes = [ctypes.c_int]
    old = L.fa_debug_set_win_bwd_grid(grid)
    try:
        out = fa.windowed_fa_backward(q, k, v, y, dy, l, m, 7)
        torch.cuda.synchronize()
    finally:
        L.fa_debug_set_win_bwd_grid(old)
    for a, r, nm in zip(out, ref, ("dq", "dk", "dv")):
        assert torch.equal(a, r), f"grid {grid} {nm}: differs from the default grid"
