"""GPU parity tests: dense backward through the C ABI (fa_dense_bwd) vs the
float64 oracle restatement of OneDFastBack (src_cpp/FlashAttention.cpp:194-252)
on the committed golden vectors, torch autograd on random shapes, and the
reference's broken cases (dv != d, Nk != N) it cannot run itself."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from conftest import assert_close, golden_files, load_golden
from oracle import fa_oracle as O

pytestmark = pytest.mark.gpu
DT = {"float32": torch.float32, "bfloat16": torch.bfloat16, "float16": torch.float16}
# gradients are sums over N terms: compare with a norm-scaled tolerance
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


def assert_grad_close(x, y, dtype, what, floor=1e-2):
    """max|x−y| and ‖x−y‖ relative to max|y| / ‖y‖, each floored at `floor`
    (gradient magnitude of O(1) inputs): dS = P(dP − D) cancels exactly in
    degenerate shapes (e.g. one key), where a pure relative check is noise."""
    x = np.asarray(x, dtype=np.float64); y = np.asarray(y, dtype=np.float64)
    assert x.shape == y.shape and np.all(np.isfinite(x)), what
    scale = max(np.abs(y).max(), floor)
    err = np.abs(x - y).max() / scale
    rel = np.linalg.norm(x - y) / max(np.linalg.norm(y), floor * np.sqrt(y.size))
    assert err <= GTOL[dtype] and rel <= GTOL[dtype], f"{what}: max err/max|y| {err:.2e}, norm rel {rel:.2e}"


def run_bwd(fa, q, k, v, do, dtype, o=None, l=None, m=None):
    Q, K, V, dO = (fa.jl_tensor(a, DT[dtype]) for a in (q, k, v, do))
    if o is None:
        Oo, l_, m_ = fa.dense_fa(Q, K, V)
    else:
        Oo = fa.jl_tensor(o, DT[dtype])
        l_ = fa.jl_tensor(np.asarray(l).reshape(-1, 1, q.shape[-1]), torch.float32)
        m_ = fa.jl_tensor(np.asarray(m).reshape(-1, 1, q.shape[-1]), torch.float32)
    dQ, dK, dV = fa.dense_fa_backward(Q, K, V, Oo, dO, l_, m_)
    torch.cuda.synchronize()
    return _np(dQ), _np(dK), _np(dV), _np(Oo)


@pytest.mark.parametrize("dtype", list(DT))
@pytest.mark.parametrize("path", golden_files("bwd_"), ids=lambda p: p.split("/")[-1][:-4])
def test_backward_golden(fa, path, dtype):
    g = load_golden(path)
    dq, dk, dv, _ = run_bwd(fa, g["q"], g["k"], g["v"], g["do"], dtype, g["o"], g["l"], g["m"])
    assert_grad_close(dq, g["dq"], dtype, "dQ")
    assert_grad_close(dk, g["dk"], dtype, "dK")
    assert_grad_close(dv, g["dv"], dtype, "dV")


@pytest.mark.parametrize("N,Nk,d,dv,B", [(64, 64, 64, 64, 2), (256, 192, 128, 128, 2), (100, 77, 12, 6, 3),
                                         (512, 512, 64, 64, 4), (1, 5, 16, 16, 1), (130, 1, 32, 8, 2),
                                         (1024, 1024, 128, 128, 1), (200, 320, 64, 128, 2),
                                         (264, 136, 128, 64, 2), (8, 8, 32, 32, 3), (72, 1000, 128, 32, 1),
                                         (1000, 8, 64, 64, 1)])
@pytest.mark.parametrize("dtype", ["float32", "bfloat16", "float16"])
def test_backward_vs_oracle_random(fa, N, Nk, d, dv, B, dtype):
    rng = np.random.default_rng(N * 31 + Nk)
    bf = lambda a: torch.tensor(a).to(torch.bfloat16).double().numpy()
    q, k = bf(rng.standard_normal((N, d, B))), bf(rng.standard_normal((Nk, d, B)))
    v, do = bf(rng.standard_normal((Nk, dv, B))), bf(rng.standard_normal((N, dv, B)))
    dq, dk, dv_, Odev = run_bwd(fa, q, k, v, do, dtype)
    # oracle on the device's O (the backward's D = rowsum(dO∘O) uses the O it is given)
    Oo, l, m = O.dense_fa3(q, k, v)
    dqr, dkr, dvr = O.dense_fa_backward(q, k, v, Odev, do, l, m)
    assert_grad_close(dq, dqr, dtype, "dQ")
    assert_grad_close(dk, dkr, dtype, "dK")
    assert_grad_close(dv_, dvr, dtype, "dV")


def test_backward_deterministic(fa):
    rng = np.random.default_rng(3)
    q, k, v, do = (fa.jl_tensor(rng.standard_normal((512, 64, 4)), torch.bfloat16) for _ in range(4))
    Oo, l, m = fa.dense_fa(q, k, v)
    a = fa.dense_fa_backward(q, k, v, Oo, do, l, m)
    b = fa.dense_fa_backward(q, k, v, Oo, do, l, m)
    torch.cuda.synchronize()
    for x, y in zip(a, b):
        assert torch.equal(x, y)


def test_backward_config4_properties(fa):
    """configs[3]: (4,16,8192,128) bf16 fwd+bwd; oracle on one slab, properties on all:
    Σ_j dS_ij = 0 ⇒ Σ_keys dK = τ Σ_q (Σ_j dS_ij) q_i = 0 (per slab, per feature)."""
    N, d, BH = 8192, 128, 64
    g = torch.Generator(device="cuda").manual_seed(5)
    mk = lambda: fa.jl_tensor(torch.randn((N, d, BH), generator=g, device="cuda"), torch.bfloat16)
    Q, K, V, dO = mk(), mk(), mk(), mk()
    Oo, l, m = fa.dense_fa(Q, K, V)
    dQ, dK, dV = fa.dense_fa_backward(Q, K, V, Oo, dO, l, m)
    torch.cuda.synchronize()
    b = 11
    sl = lambda t: _np(t[:, :, b:b + 1])
    Or, lr, mr = O.dense_fa3(sl(Q), sl(K), sl(V))
    dqr, dkr, dvr = O.dense_fa_backward(sl(Q), sl(K), sl(V), sl(Oo), sl(dO), _np(l[:, :, b:b + 1]), _np(m[:, :, b:b + 1]))
    assert_grad_close(sl(dQ), dqr, "bfloat16", "dQ")
    assert_grad_close(sl(dK), dkr, "bfloat16", "dK")
    assert_grad_close(sl(dV), dvr, "bfloat16", "dV")
    colsum = dK.float().sum(0)                       # (d, BH)
    assert float(colsum.abs().max()) <= 2e-2 * float(dK.float().abs().sum(0).max())
    # Σ_keys dV = Σ_q dO (rows of P sum to one)
    assert torch.allclose(dV.float().sum(0), dO.float().sum(0), rtol=2e-2, atol=0.5)


@pytest.mark.parametrize("N,Nk,d,dv", [(256, 256, 64, 64), (200, 136, 128, 128)])
def test_backward_fast_matches_generic(fa, N, Nk, d, dv):
    """The MFMA fast path and the generic SIMT path agree (same math, same inputs)."""
    rng = np.random.default_rng(N + d)
    Q, K, V, dO = (fa.jl_tensor(rng.standard_normal(sh), torch.bfloat16)
                   for sh in ((N, d, 2), (Nk, d, 2), (Nk, dv, 2), (N, dv, 2)))
    Oo, l, m = fa.dense_fa(Q, K, V)
    L = fa.lib()
    fast = fa.dense_fa_backward(Q, K, V, Oo, dO, l, m)
    L.fa_debug_set_bwd_generic(1)
    try:
        gen = fa.dense_fa_backward(Q, K, V, Oo, dO, l, m)
    finally:
        L.fa_debug_set_bwd_generic(0)
    torch.cuda.synchronize()
    for a, b, nm in zip(fast, gen, ("dQ", "dK", "dV")):
        assert_grad_close(_np(a), _np(b), "bfloat16", nm)


@pytest.mark.parametrize("d,dv", [(48, 48), (80, 96), (96, 32), (16, 128)])
def test_backward_head_dim_sweep(fa, d, dv):
    """Head dims outside {32, 64, 128} take the generic backward; 32/64/128
    combinations the fast one — both against the oracle."""
    rng = np.random.default_rng(d + 7 * dv)
    bf = lambda a: torch.tensor(a).to(torch.bfloat16).double().numpy()
    q, k = bf(rng.standard_normal((192, d, 2))), bf(rng.standard_normal((256, d, 2)))
    v, do = bf(rng.standard_normal((256, dv, 2))), bf(rng.standard_normal((192, dv, 2)))
    dq, dk, dv_, Odev = run_bwd(fa, q, k, v, do, "bfloat16")
    Oo, l, m = O.dense_fa3(q, k, v)
    dqr, dkr, dvr = O.dense_fa_backward(q, k, v, Odev, do, l, m)
    assert_grad_close(dq, dqr, "bfloat16", "dQ")
    assert_grad_close(dk, dkr, "bfloat16", "dK")
    assert_grad_close(dv_, dvr, "bfloat16", "dV")


@pytest.mark.parametrize("N,Nk,d,dv", [(30, 30, 12, 6), (77, 130, 64, 32), (200, 137, 96, 48),
                                       (1, 9, 8, 8), (513, 1000, 128, 80)])
@pytest.mark.parametrize("dtype", ["bfloat16", "float16"])
def test_backward_padded_fast_path(fa, N, Nk, d, dv, dtype):
    """16-bit shapes outside the MFMA kernels' (N, Nk % 8 == 0; d, dv in
    {32, 64, 128}) run them on zero-padded workspace copies: against the oracle
    and against the generic SIMT path on the same inputs (the reference test
    shape (30, 12, 6) of test/test.jl:6-10 included)."""
    tdt = torch.bfloat16 if dtype == "bfloat16" else torch.float16
    rng = np.random.default_rng(N * 3 + Nk + d)
    cast = lambda a: torch.tensor(a).to(tdt).double().numpy()
    q, k = cast(rng.standard_normal((N, d, 2))), cast(rng.standard_normal((Nk, d, 2)))
    v, do = cast(rng.standard_normal((Nk, dv, 2))), cast(rng.standard_normal((N, dv, 2)))
    Q, K, V, dO = (fa.jl_tensor(a, tdt) for a in (q, k, v, do))
    Oo, l, m = fa.dense_fa(Q, K, V)
    L = fa.lib()
    padded = fa.dense_fa_backward(Q, K, V, Oo, dO, l, m)
    L.fa_debug_set_bwd_generic(1)
    try:
        gen = fa.dense_fa_backward(Q, K, V, Oo, dO, l, m)
    finally:
        L.fa_debug_set_bwd_generic(0)
    torch.cuda.synchronize()
    dqr, dkr, dvr = O.dense_fa_backward(q, k, v, _np(Oo), do, _np(l), _np(m))
    for a, g_, r_, nm in zip(padded, gen, (dqr, dkr, dvr), ("dQ", "dK", "dV")):
        assert_grad_close(_np(a), r_, dtype, nm)
        assert_grad_close(_np(a), _np(g_), dtype, nm + " vs generic")


@pytest.mark.parametrize("N,Nk,d,dv", [(30, 30, 12, 6), (200, 137, 64, 48), (256, 256, 64, 64),
                                       (1, 70, 32, 64), (513, 300, 40, 24), (130, 200, 128, 128),
                                       (64, 64, 96, 16)])
def test_backward_f32_mfma_path(fa, N, Nk, d, dv):
    """fp32 (d, dv <= 128) runs on v_mfma_f32_32x32x2_f32 (exact fp32 products):
    against the float64 oracle at the fp32 tolerance and against the generic
    SIMT path on the same inputs."""
    rng = np.random.default_rng(N * 5 + Nk + d)
    q, k = rng.standard_normal((N, d, 2)), rng.standard_normal((Nk, d, 2))
    v, do = rng.standard_normal((Nk, dv, 2)), rng.standard_normal((N, dv, 2))
    Q, K, V, dO = (fa.jl_tensor(a, torch.float32) for a in (q, k, v, do))
    Oo, l, m = fa.dense_fa(Q, K, V)
    L = fa.lib()
    mf = fa.dense_fa_backward(Q, K, V, Oo, dO, l, m)
    L.fa_debug_set_bwd_generic(1)
    try:
        gen = fa.dense_fa_backward(Q, K, V, Oo, dO, l, m)
    finally:
        L.fa_debug_set_bwd_generic(0)
    torch.cuda.synchronize()
    dqr, dkr, dvr = O.dense_fa_backward(q, k, v, _np(Oo), do, _np(l), _np(m))
    for a, g_, r_, nm in zip(mf, gen, (dqr, dkr, dvr), ("dQ", "dK", "dV")):
        assert_grad_close(_np(a), r_, "float32", nm)
        assert_grad_close(_np(a), _np(g_), "float32", nm + " vs generic")


def _bwd_mode(fa, mode, *args, status=None):
    L = fa.lib()
    old = L.fa_debug_set_bwd_mode(mode)
    assert old >= 0
    try:
        out = fa.dense_fa_backward(*args)
        torch.cuda.synchronize()
        if status is not None:
            status.append(fa.backward_handoff_status())
    finally:
        L.fa_debug_set_bwd_mode(old)
    return out


def test_bwd_mode_knob_rejects_ablations(fa):
    """The timing-only ablation modes (wrong dQ) are compiled out of the shipped
    library: the knob refuses them and keeps the current mode."""
    L = fa.lib()
    for bad in (4, 5, 6, 7, 8, 9, 10, -1):
        assert L.fa_debug_set_bwd_mode(bad) == -1
    assert L.fa_debug_set_bwd_mode(0) == 0


@pytest.mark.parametrize("N,Nk,d,dv,B", [(512, 512, 64, 64, 2), (1024, 1024, 128, 128, 2), (1000, 520, 128, 64, 3),
                                         (256, 256, 32, 32, 4), (2048, 1024, 64, 128, 1), (513, 300, 40, 24, 2),
                                         (4096, 2048, 128, 128, 1)])
@pytest.mark.parametrize("dtype", ["bfloat16", "float16"])
def test_backward_single_pass(fa, N, Nk, d, dv, B, dtype):
    """The single-pass kernel (five MFMA products, dQ summed across the slab's
    key-block workgroups by the ordered hand-off) forced on small grids: against
    the float64 oracle and the split dK/dV + dQ passes, and bitwise reproducible."""
    tdt = torch.bfloat16 if dtype == "bfloat16" else torch.float16
    rng = np.random.default_rng(N * 7 + Nk + d + dv)
    cast = lambda a: torch.tensor(a).to(tdt).double().numpy()
    q, k = cast(rng.standard_normal((N, d, B))), cast(rng.standard_normal((Nk, d, B)))
    v, do = cast(rng.standard_normal((Nk, dv, B))), cast(rng.standard_normal((N, dv, B)))
    Q, K, V, dO = (fa.jl_tensor(a, tdt) for a in (q, k, v, do))
    Oo, l, m = fa.dense_fa(Q, K, V)
    st = []
    one = _bwd_mode(fa, 2, Q, K, V, Oo, dO, l, m, status=st)
    again = _bwd_mode(fa, 2, Q, K, V, Oo, dO, l, m, status=st)
    split = _bwd_mode(fa, 1, Q, K, V, Oo, dO, l, m, status=st)
    # the padded (513, 300, 40, 24) case runs the single pass on the padded shape too
    assert st == [0, 0, -1], st
    dqr, dkr, dvr = O.dense_fa_backward(q, k, v, _np(Oo), do, _np(l), _np(m))
    for a, a2, sp, r_, nm in zip(one, again, split, (dqr, dkr, dvr), ("dQ", "dK", "dV")):
        assert torch.equal(a, a2), nm + " not reproducible"
        assert_grad_close(_np(a), r_, dtype, nm)
        assert_grad_close(_np(a), _np(sp), dtype, nm + " vs split passes")


@pytest.mark.parametrize("d", [64, 128])
def test_backward_handoff_forms_bitwise(fa, d):
    """The single pass's two hand-off forms (sc1 write-through, and the XCD-L2-local form
    used when a slab's members share one XCD: auto at d <= 64) and the two slab
    placements (one XCD per slab, or members dealt over the chip, where the L2-local
    form does not apply) sum dQ in the same order, so dQ, dK, dV are bitwise equal;
    a chain step offset of 4 instead of 3 reorders the
    sum (other bits) and still matches the oracle.  Each form on the configs-sized grid
    (64 slabs) so the single pass and the XCD mapping are the automatic choice."""
    L = fa.lib()
    N, BH = 2048, 64
    g = torch.Generator(device="cuda").manual_seed(31 + d)
    mk = lambda: fa.jl_tensor(torch.randn((N, d, BH), generator=g, device="cuda"), torch.bfloat16)
    Q, K, V, dO = mk(), mk(), mk(), mk()
    Oo, l, m = fa.dense_fa(Q, K, V)
    outs, st = {}, {}
    old_l2, old_off, old_x = L.fa_debug_set_bwd_l2local(-1), L.fa_debug_set_bwd_hoff(3), L.fa_debug_set_bwd_xcd(-1)
    try:
        # (L2-local form, step offset, slab placement: -1 one XCD per slab, 0 chip-wide)
        for form in ((0, 3, -1), (1, 3, -1), (-1, 4, -1), (-1, 3, 0)):
            L.fa_debug_set_bwd_l2local(form[0])
            L.fa_debug_set_bwd_hoff(form[1])
            L.fa_debug_set_bwd_xcd(form[2])
            outs[form] = [t.clone() for t in fa.dense_fa_backward(Q, K, V, Oo, dO, l, m)]
            st[form] = fa.backward_handoff_status()
    finally:
        L.fa_debug_set_bwd_l2local(old_l2)
        L.fa_debug_set_bwd_hoff(old_off)
        L.fa_debug_set_bwd_xcd(old_x)
    assert all(v == 0 for v in st.values()), st
    for a, b_, c_, nm in zip(outs[(0, 3, -1)], outs[(1, 3, -1)], outs[(-1, 3, 0)], ("dQ", "dK", "dV")):
        assert torch.equal(a, b_), nm + ": L2-local hand-off not bitwise equal to sc1"
        assert torch.equal(a, c_), nm + ": members dealt chip-wide not bitwise equal to one XCD per slab"
    b = 17
    sl = lambda t: _np(t[:, :, b:b + 1])
    dqr, dkr, dvr = O.dense_fa_backward(sl(Q), sl(K), sl(V), sl(Oo), sl(dO), _np(l[:, :, b:b + 1]),
                                        _np(m[:, :, b:b + 1]))
    for form in outs:
        for a, r_, nm in zip(outs[form], (dqr, dkr, dvr), ("dQ", "dK", "dV")):
            assert_grad_close(sl(a), r_, "bfloat16", f"{nm} form {form}")


def test_backward_single_pass_fallback(fa):
    """A hand-off timeout (forced: the timeout word starts set) leaves dK, dV of the
    single pass and recomputes dQ in the guarded dQ pass: the result still matches."""
    rng = np.random.default_rng(17)
    N, d, B = 1024, 128, 2
    Q, K, V, dO = (fa.jl_tensor(rng.standard_normal((N, d, B)), torch.bfloat16) for _ in range(4))
    Oo, l, m = fa.dense_fa(Q, K, V)
    st = []
    fb = _bwd_mode(fa, 3, Q, K, V, Oo, dO, l, m, status=st)
    sp = _bwd_mode(fa, 1, Q, K, V, Oo, dO, l, m, status=st)
    assert st == [1, -1], st          # the timeout is reported
    for a, b_, nm in zip(fb, sp, ("dQ", "dK", "dV")):
        assert_grad_close(_np(a), _np(b_), "bfloat16", nm + " (fallback) vs split passes")


def test_backward_handoff_status_errors(fa):
    """The status query refuses a workspace that no backward wrote a header into."""
    rng = np.random.default_rng(2)
    Q, K, V = (fa.jl_tensor(rng.standard_normal((256, 64, 2)), torch.bfloat16) for _ in range(3))
    fa.windowed_fa(fa.jl_tensor(rng.standard_normal((16, 16, 64, 1)), torch.bfloat16),
                   fa.jl_tensor(rng.standard_normal((16, 16, 64, 1)), torch.bfloat16),
                   fa.jl_tensor(rng.standard_normal((16, 16, 64, 1)), torch.bfloat16), 4)
    Oo, l, m = fa.dense_fa(Q, K, V)
    fa.dense_fa_backward(Q, K, V, Oo, Oo, l, m)
    assert fa.backward_handoff_status() in (-1, 0)
    L = fa.lib()
    junk = torch.zeros(1024, dtype=torch.uint8, device="cuda")
    st = __import__("ctypes").c_int(5)
    rc = L.fa_dense_bwd_handoff_status(fa._ptr(junk), 1024, None, __import__("ctypes").byref(st))
    assert rc == fa.FA_ERR_INVALID_ARG and st.value == 5


def test_backward_two_streams_concurrent(fa):
    """Two configs[3]-sized backward calls (N 8192, d 128, 64 slabs) on two streams at
    once, each holding CUs the other's single pass would use.  Every hand-off wait of
    the single pass is on a member of lower launch id (two chains per slice, cut where
    the rotated order wraps: fa_bwd.hip bwd_fused), so neither call can strand: both
    must complete their hand-off (status 0 on every concurrent call, no slab given up
    and recomputed) and match the float64 oracle on one slab each.  Timing is reported,
    and bounded only loosely (2.5x the same pair back to back on one stream, against
    ~7x for round 3's stalled chains): the mechanism is what the test asserts, not a
    ratio within the 5-7 % box-to-box variance."""
    import time
    N, d, BH = 8192, 128, 64
    g = torch.Generator(device="cuda").manual_seed(23)
    mk = lambda: fa.jl_tensor(torch.randn((N, d, BH), generator=g, device="cuda"), torch.bfloat16)
    ins = []
    for _ in range(2):
        Q, K, V, dO = mk(), mk(), mk(), mk()
        Oo, l, m = fa.dense_fa(Q, K, V)
        ins.append((Q, K, V, Oo, dO, l, m))
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]

    def pair(concurrent):
        outs = [None, None]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(2):
            with torch.cuda.stream(streams[i if concurrent else 0]):
                outs[i] = fa.dense_fa_backward(*ins[i])
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        status = []
        for i in range(2 if concurrent else 1):
            with torch.cuda.stream(streams[i]):
                status.append(fa.backward_handoff_status())
        return outs, status, dt

    pair(False); pair(True)   # warm up (allocations, code objects, clocks)
    runs = []
    for _ in range(3):   # interleaved repetitions
        runs.append((pair(False), pair(True)))
    serial = sorted(r[0][2] for r in runs)[1]
    conc = sorted(r[1][2] for r in runs)[1]
    print(f"two-stream backward: serial pair {[round(r[0][2] * 1e3, 2) for r in runs]} ms, concurrent pair "
          f"{[round(r[1][2] * 1e3, 2) for r in runs]} ms, hand-off status {[r[1][1] for r in runs]}")
    assert all(r[0][1] == [0] and r[1][1] == [0, 0] for r in runs), [(r[0][1], r[1][1]) for r in runs]
    assert conc <= 2.5 * serial, f"concurrent pair {conc * 1e3:.2f} ms vs serial {serial * 1e3:.2f} ms (medians)"
    outs = runs[-1][1][0]
    for i, b in ((0, 5), (1, 40)):
        Q, K, V, Oo, dO, l, m = ins[i]
        sl = lambda t: _np(t[:, :, b:b + 1])
        dqr, dkr, dvr = O.dense_fa_backward(sl(Q), sl(K), sl(V), sl(Oo), sl(dO),
                                            _np(l[:, :, b:b + 1]), _np(m[:, :, b:b + 1]))
        for a, r_, nm in zip(outs[i], (dqr, dkr, dvr), ("dQ", "dK", "dV")):
            assert_grad_close(sl(a), r_, "bfloat16", f"stream {i} {nm}")


@pytest.mark.parametrize("N,Nk,d,BH,xcd", [(16384, 16384, 128, 64, -1), (8192, 6144, 128, 96, 0),
                                          (4096, 3072, 64, 200, -1)])
def test_backward_single_pass_multipass_grid_solo(fa, N, Nk, d, BH, xcd):
    """Solo calls whose single-pass grid takes several passes over the chip (64 members x
    64 slabs = 16 passes; 24 members — not a divisor of the CUs — dealt chip-wide, forced;
    12 members x 200 slabs) complete the hand-off (status 0: no slab gives up while the
    launch still dispatches), and dQ is bitwise reproducible."""
    L = fa.lib()
    g = torch.Generator(device="cuda").manual_seed(N + Nk + BH)
    mk = lambda n: fa.jl_tensor(torch.randn((n, d, BH), generator=g, device="cuda"), torch.bfloat16)
    Q, K, V, dO = mk(N), mk(Nk), mk(Nk), mk(N)
    Oo, l, m = fa.dense_fa(Q, K, V)
    old_x = L.fa_debug_set_bwd_xcd(xcd)
    try:
        st = []
        one = _bwd_mode(fa, 2, Q, K, V, Oo, dO, l, m, status=st)
        one = [t.clone() for t in one]
        again = _bwd_mode(fa, 2, Q, K, V, Oo, dO, l, m, status=st)
    finally:
        L.fa_debug_set_bwd_xcd(old_x)
    assert st == [0, 0], st
    for a, b_, nm in zip(one, again, ("dQ", "dK", "dV")):
        assert torch.equal(a, b_), nm + " not reproducible"
    b = BH - 1
    sl = lambda t: _np(t[:, :, b:b + 1])
    dqr, dkr, dvr = O.dense_fa_backward(sl(Q), sl(K), sl(V), sl(Oo), sl(dO), _np(l[:, :, b:b + 1]),
                                        _np(m[:, :, b:b + 1]))
    for a, r_, nm in zip(one, (dqr, dkr, dvr), ("dQ", "dK", "dV")):
        assert_grad_close(sl(a), r_, "bfloat16", nm)


@pytest.mark.parametrize("N,Nk,d,dv,BH", [(2048, 2048, 64, 64, 64), (4096, 2048, 128, 128, 32),
                                          (1024, 768, 128, 64, 40)])
def test_backward_chain_b_combine_bitwise(fa, N, Nk, d, dv, BH):
    """Where a slice's member order wraps it runs as two chains, and dQ = A + B is made
    either by chain B's tail (A done at its poll: every slice of a solo call) or, when
    A finished later, by the guarded dQ pass after the launch (fused_combine) — the
    path a co-tenant can force on any slice.  Forced for every wrapped slice
    (fa_debug_set_bwd_nodirect), it must give the same bits, since it is the same single
    fp32 add; header word 3 shows the combine ran."""
    import ctypes
    L = fa.lib()
    L.fa_debug_set_bwd_nodirect.restype = ctypes.c_int
    g = torch.Generator(device="cuda").manual_seed(N + d + BH)
    mk = lambda n, c: fa.jl_tensor(torch.randn((n, c, BH), generator=g, device="cuda"), torch.bfloat16)
    Q, K, V, dO = mk(N, d), mk(Nk, d), mk(Nk, dv), mk(N, dv)
    Oo, l, m = fa.dense_fa(Q, K, V)
    st, comb = [], []
    old = L.fa_debug_set_bwd_nodirect(1)
    assert old == 0
    try:
        forced = [t.clone() for t in _bwd_mode(fa, 2, Q, K, V, Oo, dO, l, m, status=st)]
        comb.append(fa._backward_header_word(3))
    finally:
        assert L.fa_debug_set_bwd_nodirect(old) == 1
    assert L.fa_debug_set_bwd_nodirect(2) == -2
    direct = [t.clone() for t in _bwd_mode(fa, 2, Q, K, V, Oo, dO, l, m, status=st)]
    comb.append(fa._backward_header_word(3))
    assert st == [0, 0], st
    assert comb[0] == 1, "the forced run never reached the combine"
    for a, b_, nm in zip(forced, direct, ("dQ", "dK", "dV")):
        assert torch.equal(a, b_), nm + ": combine in the dQ pass not bitwise equal to chain B's direct add"
    b = BH // 2
    sl = lambda t: _np(t[:, :, b:b + 1])
    dqr, dkr, dvr = O.dense_fa_backward(sl(Q), sl(K), sl(V), sl(Oo), sl(dO), _np(l[:, :, b:b + 1]),
                                        _np(m[:, :, b:b + 1]))
    for a, r_, nm in zip(forced, (dqr, dkr, dvr), ("dQ", "dK", "dV")):
        assert_grad_close(sl(a), r_, "bfloat16", nm)
