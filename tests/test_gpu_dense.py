"""GPU parity tests: dense forward through the C ABI (fa_dense_fwd) vs the
float64 oracle (oracle/fa_oracle.py) on the committed golden vectors, edge
cases the reference exercises or breaks on, and size-independent properties
at BASELINE.json's full sizes.  Tolerances: tests/conftest.py."""
from __future__ import annotations

import math

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


@pytest.mark.parametrize("dtype", list(DT))
@pytest.mark.parametrize("path", golden_files("dense_"), ids=lambda p: p.split("/")[-1][:-4])
def test_dense_golden(fa, path, dtype):
    g = load_golden(path)
    q, k, v = (fa.jl_tensor(g[x], DT[dtype]) for x in ("q", "k", "v"))
    y, l, m = fa.dense_fa(q, k, v)
    torch.cuda.synchronize()
    assert tuple(y.shape) == g["y"].shape and fa.is_jl_contiguous(y)
    assert_close(_np(y), g["y"], dtype, "y")
    assert_lm_close(_np(l), g["l"], dtype, "l")
    assert_lm_close(_np(m), g["m"], dtype, "m")


def test_reference_test_jl_shape_against_dpa(fa):
    """test/test.jl:5-21: dense_fa ≈ dense_dpa with Nq = Nkv = 30, dqk = 12, dv = 6
    (the reference itself throws DimensionMismatch here, Appendix A.1)."""
    rng = np.random.default_rng(0)
    q, k, v = rng.random((30, 12, 2)), rng.random((30, 12, 2)), rng.random((30, 6, 2))
    y, l, m = fa.dense_fa(*(fa.jl_tensor(a, torch.float32) for a in (q, k, v)))
    y1, _ = O.dense_dpa(q.astype(np.float32), k.astype(np.float32), v.astype(np.float32))
    # Julia ≈ : norm(x - y) <= sqrt(eps(T)) * max(norm(x), norm(y))
    assert np.linalg.norm(_np(y) - y1) <= math.sqrt(np.finfo(np.float32).eps) * np.linalg.norm(y1)


def test_inplace_overwrites_every_output(fa):
    """dense_fa! semantics: callee initialises O, l, m (src/dense.jl:58-60)."""
    rng = np.random.default_rng(1)
    N, Nk, d, dv, B = 200, 190, 64, 64, 3
    q, k, v = rng.standard_normal((N, d, B)), rng.standard_normal((Nk, d, B)), rng.standard_normal((Nk, dv, B))
    Q, K, V = (fa.jl_tensor(a, torch.bfloat16) for a in (q, k, v))
    Ob = fa.jl_empty((N, dv, B), torch.bfloat16); Ob.fill_(float("nan"))
    lb = fa.jl_empty((N, 1, B)); lb.fill_(float("nan"))
    mb = fa.jl_empty((N, 1, B)); mb.fill_(float("nan"))
    r = fa.dense_fa_(Ob, lb, mb, Q, K, V)
    assert r[0] is Ob and r[1] is lb and r[2] is mb
    torch.cuda.synchronize()
    yr, lr, mr = O.dense_fa3(_np(Q), _np(K), _np(V))
    assert_close(_np(Ob), yr, "bfloat16", "O")
    assert_lm_close(_np(lb), lr, "bfloat16", "l")
    assert_lm_close(_np(mb), mr, "bfloat16", "m")


@pytest.mark.parametrize("N,Nk,d,dv,B", [(1, 1, 64, 64, 1), (1, 300, 64, 64, 2), (300, 1, 64, 64, 2),
                                         (65, 63, 16, 8, 2), (129, 257, 128, 128, 1), (127, 65, 128, 32, 2),
                                         (33, 4100, 64, 64, 1), (3, 7, 1, 1, 2), (70, 70, 33, 65, 1)])
@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
def test_ragged_and_tiny_shapes(fa, N, Nk, d, dv, B, dtype):
    """Ragged N / Nk (keys masked to -inf, not zero-filled: Appendix A.4),
    Nk != N and dv != d (lifted reference restrictions), head-dim padding."""
    rng = np.random.default_rng(N * 1000 + Nk)
    bf = lambda a: torch.tensor(a).to(torch.bfloat16).double().numpy()
    q, k, v = bf(rng.standard_normal((N, d, B))), bf(rng.standard_normal((Nk, d, B))), bf(rng.standard_normal((Nk, dv, B)))
    y, l, m = fa.dense_fa(*(fa.jl_tensor(a, DT[dtype]) for a in (q, k, v)))
    yr, lr, mr = O.dense_fa3(q, k, v)
    torch.cuda.synchronize()
    assert_close(_np(y), yr, dtype, "y")
    assert_lm_close(_np(l), lr, dtype, "l")
    assert_lm_close(_np(m), mr, dtype, "m")


@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
def test_running_max_rescale_branch(fa, dtype):
    """Force the online-softmax rescale at chosen tiles (cdna guide rule 26):
    a spike key whose score jumps far above every earlier tile's max, placed
    in the 3rd and 9th key tiles, for a subset of query rows."""
    rng = np.random.default_rng(7)
    N, Nk, d, B = 256, 640, 64, 2
    q = rng.standard_normal((N, d, B)) * 0.5
    k = rng.standard_normal((Nk, d, B)) * 0.5
    v = rng.standard_normal((Nk, d, B))
    k[150] = q[10] * 6.0
    k[560] = q[200] * 8.0
    k[600, :, 1] = -q[100, :, 1] * 8.0
    bf = lambda a: torch.tensor(a).to(torch.bfloat16).double().numpy()
    q, k, v = bf(q), bf(k), bf(v)
    y, l, m = fa.dense_fa(*(fa.jl_tensor(a, DT[dtype]) for a in (q, k, v)))
    yr, lr, mr = O.dense_fa3(q, k, v)
    torch.cuda.synchronize()
    assert_close(_np(y), yr, dtype, "y")
    assert_lm_close(_np(m), mr, dtype, "m")
    assert_lm_close(_np(l), lr, dtype, "l")


def test_explicit_scale_and_nondefault_stream(fa):
    rng = np.random.default_rng(9)
    N, d, B = 130, 32, 2
    q, k, v = (rng.standard_normal((N, d, B)) for _ in range(3))
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        y, l, m = fa.dense_fa(*(fa.jl_tensor(a, torch.float32) for a in (q, k, v)), scale=0.3)
    s.synchronize()
    # reference math with tau replaced by 0.3 ≡ oracle on q scaled by 0.3*sqrt(d)
    yr, lr, mr = O.dense_fa3(q * 0.3 * math.sqrt(d), k, v)
    assert_close(_np(y), yr, "float32", "y")
    assert_lm_close(_np(m), mr, "float32", "m")


def test_deterministic(fa):
    rng = np.random.default_rng(10)
    q, k, v = (fa.jl_tensor(rng.standard_normal((1000, 64, 4)), torch.bfloat16) for _ in range(3))
    a = fa.dense_fa(q, k, v)
    b = fa.dense_fa(q, k, v)
    torch.cuda.synchronize()
    for x, y in zip(a, b):
        assert torch.equal(x, y)


def _full_size_properties(fa, N, d, BH, dtype, check_slabs=(0,), rows=None):
    """BASELINE config at full size: oracle on a few slabs (all query rows, or
    the query-row ranges `rows` against ALL keys) + size-independent
    properties on all slabs."""
    g = torch.Generator(device="cuda").manual_seed(1)
    Q = fa.jl_empty((N, d, BH), dtype); Q.copy_(torch.randn(Q.shape, generator=g, device="cuda"))
    K = fa.jl_empty((N, d, BH), dtype); K.copy_(torch.randn(K.shape, generator=g, device="cuda"))
    V = fa.jl_empty((N, d, BH), dtype); V.copy_(torch.randn(V.shape, generator=g, device="cuda"))
    y, l, m = fa.dense_fa(Q, K, V)
    torch.cuda.synchronize()
    # (1) oracle on selected slabs
    for b in check_slabs:
        Kb, Vb = _np(K[:, :, b:b + 1]), _np(V[:, :, b:b + 1])
        for r0, r1 in (rows or [(0, N)]):
            yr, lr, mr = O.dense_fa3(_np(Q[r0:r1, :, b:b + 1]), Kb, Vb)
            assert_close(_np(y[r0:r1, :, b:b + 1]), yr, "bfloat16", f"y slab {b} rows {r0}:{r1}")
            assert_lm_close(_np(l[r0:r1, :, b:b + 1]), lr, "bfloat16", f"l slab {b}")
            assert_lm_close(_np(m[r0:r1, :, b:b + 1]), mr, "bfloat16", f"m slab {b}")
    yf = y.float()
    # (2) convex combination: min_j V <= O <= max_j V per feature and slab
    vmin = V.float().amin(0, keepdim=True); vmax = V.float().amax(0, keepdim=True)
    tol = 1e-2 * (1 + vmax.abs())
    assert bool(((yf >= vmin - tol) & (yf <= vmax + tol)).all())
    # (3) 1 <= l <= Nk
    assert bool(((l >= 1 - 1e-4) & (l <= N * (1 + 1e-4))).all())
    # (4) affine equivariance: softmax rows sum to one, so V -> 2V + 1 gives 2O + 1
    V2 = fa.jl_empty(V.shape, dtype); V2.copy_(2 * V.float() + 1)
    y2, _, m2 = fa.dense_fa(Q, K, V2)
    torch.cuda.synchronize()
    assert torch.allclose(y2.float(), 2 * yf + 1, atol=4e-2, rtol=2e-2)
    assert torch.equal(m2, m)
    # (5) key permutation invariance (K and V tokens permuted together)
    perm = torch.randperm(N, generator=torch.Generator().manual_seed(3)).cuda()
    Kp = fa.jl_empty(K.shape, dtype); Kp.copy_(K[perm])
    Vp = fa.jl_empty(V.shape, dtype); Vp.copy_(V[perm])
    y3, l3, m3 = fa.dense_fa(Q, Kp, Vp)
    torch.cuda.synchronize()
    assert torch.allclose(y3.float(), yf, atol=2e-2, rtol=2e-2)
    assert torch.allclose(m3, m, atol=1e-5, rtol=1e-5)
    assert torch.allclose(l3, l, rtol=1e-4)


def test_config2_full_size_properties(fa):
    """BASELINE configs[1]: (B,H,N,d) = (4,16,4096,64) bf16 → (N, d, B·H) = (4096, 64, 64)."""
    _full_size_properties(fa, 4096, 64, 64, torch.bfloat16, check_slabs=(0, 37, 63))


def test_config4_full_size_forward_properties(fa):
    """BASELINE configs[3] forward: (4,16,8192,128) bf16 → (8192, 128, 64)."""
    _full_size_properties(fa, 8192, 128, 64, torch.bfloat16, check_slabs=(5,))


def test_config5_per_gpu_share_forward(fa):
    """BASELINE configs[4]: (B,H,N,d) = (64,16,16384,128) bf16 sharded over
    (B·H) on 8 GPUs -> one GPU's share is 128 slabs of (16384, 128).  The oracle
    on the first and last 256 query rows (all 16384 keys) of slabs 0 and 127,
    size-independent properties on all 128 slabs."""
    _full_size_properties(fa, 16384, 128, 128, torch.bfloat16, check_slabs=(0, 127),
                          rows=[(0, 256), (16384 - 256, 16384)])


def test_config5_shard_views_match_unsharded(fa):
    """The sharded call (fa_hip.shard.local_slabs: zero-copy views of each
    rank's contiguous slab range) gives bitwise the unsharded result, for the
    configs[4] head dim split over 8 ranks at reduced N (shards large enough
    that neither call takes the small-grid split-KV kernels, whose fp32
    partial combine is not bitwise the unsplit order)."""
    from fa_hip.shard import local_slabs
    N, d, BH, world = 4096, 128, 256, 8
    g = torch.Generator(device="cuda").manual_seed(21)
    Q, K, V = (fa.jl_empty((N, d, BH), torch.bfloat16) for _ in range(3))
    for t in (Q, K, V):
        t.normal_(generator=g)
    y, l, m = fa.dense_fa(Q, K, V)
    for r in range(world):
        q, k, v = (local_slabs(t, world, r) for t in (Q, K, V))
        assert fa.is_jl_contiguous(q)
        yr, lr, mr = fa.dense_fa(q, k, v)
        a = r * BH // world
        assert torch.equal(yr, y[..., a:a + BH // world])
        assert torch.equal(mr, m[..., a:a + BH // world]) and torch.equal(lr, l[..., a:a + BH // world])


def test_lazy_rescale_accuracy_cost(fa):
    """The forward's lazy rescale (kRescaleLog2 = 8: P may reach 2^8 before it is
    quantised to bf16, cdna guide T13) against the textbook order (threshold 0,
    fa_debug_set_rescale_threshold) on inputs whose running max climbs
    steadily over the key sweep, so the deferred max lags the true max by up to
    8 log2 units on most tiles.  Both vs the float64 oracle: the threshold-8
    error stays within the bf16 tolerance and within a small factor of the
    threshold-0 error (DESIGN.md §3 states the measured numbers)."""
    L = fa.lib()
    rng = np.random.default_rng(17)
    N, Nk, d, B = 128, 4096, 64, 2
    u = rng.standard_normal(d); u /= np.linalg.norm(u)
    q = np.repeat((u * 8.0)[None, :, None], N, 0).repeat(B, 2) + 0.3 * rng.standard_normal((N, d, B))
    # raw score of key j ~ 8 * t_j with t_j rising by 60 natural-log units (x sqrt(d) / 8)
    t = np.linspace(-1.0, 1.0, Nk) * 60.0 * math.sqrt(d) / 8.0 / 2.0
    k = t[:, None, None] * u[None, :, None] + 0.3 * rng.standard_normal((Nk, d, B))
    v = rng.uniform(-4, 4, (Nk, d, B))
    bf = lambda a: torch.tensor(a).to(torch.bfloat16).double().numpy()
    q, k, v = bf(q), bf(k), bf(v)
    yr, lr, mr = O.dense_fa3(q, k, v)
    errs = {}
    for thr in (8.0, 0.0):
        old = L.fa_debug_set_rescale_threshold(thr)
        try:
            y, l, m = fa.dense_fa(*(fa.jl_tensor(a, torch.bfloat16) for a in (q, k, v)))
            torch.cuda.synchronize()
        finally:
            L.fa_debug_set_rescale_threshold(old)
        assert_close(_np(y), yr, "bfloat16", f"y threshold {thr}")
        assert_lm_close(_np(m), mr, "bfloat16", "m")
        assert_lm_close(_np(l), lr, "bfloat16", "l")
        errs[thr] = float(np.abs(_np(y) - yr).max())
    print(f"lazy rescale max |y - oracle|: threshold 8 {errs[8.0]:.3e}, threshold 0 {errs[0.0]:.3e}")
    assert errs[8.0] <= 1.5e-2
    assert errs[8.0] <= 6.0 * errs[0.0] + 1e-3


def test_workspace_per_stream(fa):
    """Concurrent calls on two streams that both need scratch (ragged Nk: padded
    K / V copies) get separate workspaces and correct results."""
    rng = np.random.default_rng(33)
    shapes = [(300, 1001, 64, 64, 3), (500, 777, 128, 64, 2)]
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    ins, outs = [], []
    for (N, Nk, d, dv, B) in shapes:
        bf = lambda a: torch.tensor(a).to(torch.bfloat16).double().numpy()
        ins.append((bf(rng.standard_normal((N, d, B))), bf(rng.standard_normal((Nk, d, B))),
                    bf(rng.standard_normal((Nk, dv, B)))))
    dev = [tuple(fa.jl_tensor(a, torch.bfloat16) for a in x) for x in ins]
    torch.cuda.synchronize()
    for _ in range(3):
        outs = []
        for st, x in zip((s1, s2), dev):
            with torch.cuda.stream(st):
                outs.append(fa.dense_fa(*x))
        torch.cuda.synchronize()
    keys = [k for k in fa._WS if k[2] in (s1.cuda_stream, s2.cuda_stream)]
    assert len(keys) == 2 and fa._WS[keys[0]].data_ptr() != fa._WS[keys[1]].data_ptr()
    for (q, k, v), (y, l, m) in zip(ins, outs):
        yr, lr, mr = O.dense_fa3(q, k, v)
        assert_close(_np(y), yr, "bfloat16", "y")
        assert_lm_close(_np(m), mr, "bfloat16", "m")


def test_misaligned_kv_takes_padded_fast_path(fa):
    """K / V views that are not 16-B aligned with Nk % 8 == 0: the mirror adds
    room for the padded copies and the fast kernels run on them; the result
    matches the oracle and the aligned call bitwise."""
    rng = np.random.default_rng(44)
    N, Nk, d, B = 256, 512, 64, 2
    bf = lambda a: torch.tensor(a).to(torch.bfloat16).double().numpy()
    q, k, v = bf(rng.standard_normal((N, d, B))), bf(rng.standard_normal((Nk, d, B))), bf(rng.standard_normal((Nk, d, B)))
    Q, K, V = (fa.jl_tensor(a, torch.bfloat16) for a in (q, k, v))
    def shifted(t):
        raw = torch.empty(t.numel() + 1, dtype=t.dtype, device=t.device)
        view = raw[1:].as_strided(tuple(t.shape), fa.jl_strides(t.shape))
        view.copy_(t)
        assert view.data_ptr() % 16 != 0
        return view
    Ks, Vs = shifted(K), shifted(V)
    y1, l1, m1 = fa.dense_fa(Q, Ks, Vs)
    y0, l0, m0 = fa.dense_fa(Q, K, V)
    torch.cuda.synchronize()
    yr, lr, mr = O.dense_fa3(q, k, v)
    assert_close(_np(y1), yr, "bfloat16", "y misaligned")
    assert torch.equal(y1, y0) and torch.equal(m1, m0) and torch.equal(l1, l0)


@pytest.mark.parametrize("d,dv", [(8, 8), (24, 40), (48, 48), (56, 72), (80, 80), (96, 64), (104, 120), (112, 112), (120, 24)])
@pytest.mark.parametrize("dtype", ["bfloat16", "float16"])
def test_head_dim_sweep_fast_path(fa, d, dv, dtype):
    """Head dims that are not 32/64/128 run the fast kernels zero-padded to the next
    class (aligned N, Nk: the fast path), for d != dv in both directions."""
    rng = np.random.default_rng(d * 131 + dv)
    rd = lambda a: torch.tensor(a).to(DT[dtype]).double().numpy()
    q, k, v = rd(rng.standard_normal((256, d, 2))), rd(rng.standard_normal((320, d, 2))), rd(rng.standard_normal((320, dv, 2)))
    y, l, m = fa.dense_fa(*(fa.jl_tensor(a, DT[dtype]) for a in (q, k, v)))
    torch.cuda.synchronize()
    yr, lr, mr = O.dense_fa3(q, k, v)
    assert_close(_np(y), yr, dtype, "y")
    assert_lm_close(_np(l), lr, dtype, "l")
    assert_lm_close(_np(m), mr, dtype, "m")


def test_long_single_slab(fa):
    """One slab with N = Nk = 65536 (512 key tiles, 128 query blocks): the oracle
    on the first and last query blocks (K, V over the whole sequence)."""
    N, d = 65536, 64
    g = torch.Generator(device="cuda").manual_seed(11)
    Q, K, V = (fa.jl_empty((N, d, 1), torch.bfloat16) for _ in range(3))
    for t in (Q, K, V):
        t.copy_(torch.randn((N, d, 1), generator=g, device="cuda"))
    y, l, m = fa.dense_fa(Q, K, V)
    torch.cuda.synchronize()
    Kh, Vh = _np(K), _np(V)
    for r0 in (0, N - 128):
        yr, lr, mr = O.dense_fa3(_np(Q[r0:r0 + 128]), Kh, Vh)
        assert_close(_np(y[r0:r0 + 128]), yr, "bfloat16", f"y[{r0}]")
        assert_lm_close(_np(l[r0:r0 + 128]), lr, "bfloat16", "l")
        assert_lm_close(_np(m[r0:r0 + 128]), mr, "bfloat16", "m")


@pytest.mark.parametrize("N,Nk,d,dv", [(30, 30, 12, 6), (77, 130, 64, 32), (1000, 1001, 96, 48),
                                       (257, 4095, 128, 128), (64, 9, 64, 64)])
@pytest.mark.parametrize("dtype", ["bfloat16", "float16"])
def test_forward_padded_keys_path(fa, N, Nk, d, dv, dtype):
    """Ragged Nk through fa_dense_fwd_ws (zero-padded K / V copies, fast kernels)
    against the oracle and against fa_dense_fwd without a workspace (generic kernel)."""
    import ctypes
    tdt = DT[dtype]
    rng = np.random.default_rng(N + Nk + d)
    cast = lambda a: torch.tensor(a).to(tdt).double().numpy()
    q, k, v = cast(rng.standard_normal((N, d, 2))), cast(rng.standard_normal((Nk, d, 2))), cast(rng.standard_normal((Nk, dv, 2)))
    Q, K, V = (fa.jl_tensor(a, tdt) for a in (q, k, v))
    L = fa.lib()
    code = fa._dtype_code(Q)
    assert L.fa_dense_fwd_workspace(code, N, Nk, d, dv, 2) > 0
    y1, l1, m1 = fa.dense_fa(Q, K, V)                     # workspace path
    y2 = fa.jl_empty((N, dv, 2), tdt); l2 = fa.jl_empty((N, 1, 2)); m2 = fa.jl_empty((N, 1, 2))
    P = lambda t: ctypes.c_void_p(t.data_ptr())
    assert L.fa_dense_fwd(code, P(Q), P(K), P(V), P(y2), P(l2), P(m2), N, Nk, d, dv, 2, 0.0,
                          ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)) == 0
    torch.cuda.synchronize()
    yr, lr, mr = O.dense_fa3(q, k, v)
    assert_close(_np(y1), yr, dtype, "y (padded keys)")
    assert_lm_close(_np(l1), lr, dtype, "l")
    assert_lm_close(_np(m1), mr, dtype, "m")
    assert_close(_np(y1), _np(y2), dtype, "y padded vs generic")


@pytest.mark.parametrize("N,Nk,d,dv,B", [(512, 512, 64, 64, 1), (4096, 4096, 64, 64, 1), (128, 32768, 128, 128, 2),
                                         (1000, 3001, 96, 48, 1), (33, 4096, 32, 64, 3), (16384, 2048, 64, 64, 1)])
def test_forward_split_kv(fa, N, Nk, d, dv, B):
    """Small grids split the key range over workgroups (fp32 partials + an
    ordered combine): against the oracle on every slab, and against the unsplit
    kernel (fa_dense_fwd without a workspace) on the same inputs."""
    import ctypes
    rng = np.random.default_rng(N + Nk + d + B)
    bf = lambda a: torch.tensor(a).to(torch.bfloat16).double().numpy()
    q, k, v = bf(rng.standard_normal((N, d, B))), bf(rng.standard_normal((Nk, d, B))), bf(rng.standard_normal((Nk, dv, B)))
    Q, K, V = (fa.jl_tensor(a, torch.bfloat16) for a in (q, k, v))
    L = fa.lib()
    assert L.fa_dense_fwd_workspace(fa._dtype_code(Q), N, Nk, d, dv, B) > 0, "expected a split plan"
    y1, l1, m1 = fa.dense_fa(Q, K, V)
    y2 = fa.jl_empty((N, dv, B), torch.bfloat16); l2 = fa.jl_empty((N, 1, B)); m2 = fa.jl_empty((N, 1, B))
    P = lambda t: ctypes.c_void_p(t.data_ptr())
    assert L.fa_dense_fwd(fa._dtype_code(Q), P(Q), P(K), P(V), P(y2), P(l2), P(m2), N, Nk, d, dv, B, 0.0,
                          ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)) == 0
    torch.cuda.synchronize()
    if N * Nk <= 4096 * 4096:
        yr, lr, mr = O.dense_fa3(q, k, v)
        assert_close(_np(y1), yr, "bfloat16", "y split")
        assert_lm_close(_np(l1), lr, "bfloat16", "l split")
        assert_lm_close(_np(m1), mr, "bfloat16", "m split")
    assert_close(_np(y1), _np(y2), "bfloat16", "y split vs unsplit")
    assert np.array_equal(_np(m1), _np(m2)), "m is the exact row max either way"
    assert_lm_close(_np(l1), _np(l2), "bfloat16", "l split vs unsplit")


@pytest.mark.parametrize("variant", [5, 7, 20, 30])
@pytest.mark.parametrize("N,Nk,d,dv,B,dtype", [(300, 200, 64, 64, 2, "bfloat16"), (513, 4100, 64, 32, 1, "bfloat16"),
                                               (256, 320, 128, 128, 2, "bfloat16"), (100, 72, 32, 64, 3, "float16"),
                                               (77, 136, 128, 64, 1, "float16"), (1024, 1024, 96, 96, 1, "bfloat16")])
def test_forced_forward_variants(fa, variant, N, Nk, d, dv, B, dtype):
    """Every fast-kernel geometry (fa_debug_set_fwd_variant: 5, 7 the 8-wave 32x32x16
    kernels, 20 the defaults with per-element Q / O accesses, 30 the one-wave-per-SIMD
    persistent kernel where its shape rules allow, the defaults elsewhere) against the
    oracle, ragged Nk and dv != d included."""
    L = fa.lib()
    rng = np.random.default_rng(N * 7 + Nk + d * 3 + dv)
    cast = lambda a: torch.tensor(a).to(DT[dtype]).double().numpy()
    q, k, v = cast(rng.standard_normal((N, d, B))), cast(rng.standard_normal((Nk, d, B))), cast(rng.standard_normal((Nk, dv, B)))
    old = L.fa_debug_set_fwd_variant(variant)
    try:
        y, l, m = fa.dense_fa(*(fa.jl_tensor(a, DT[dtype]) for a in (q, k, v)))
        torch.cuda.synchronize()
    finally:
        L.fa_debug_set_fwd_variant(old)
    yr, lr, mr = O.dense_fa3(q, k, v)
    assert_close(_np(y), yr, dtype, f"y variant {variant}")
    assert_lm_close(_np(l), lr, dtype, "l")
    assert_lm_close(_np(m), mr, dtype, "m")


@pytest.mark.parametrize("N,Nk,d,dv,B", [(4096, 4096, 64, 64, 32), (1000, 520, 64, 32, 128), (8, 64, 32, 32, 2),
                                         (776, 1024, 128, 128, 64), (264, 200, 128, 64, 128), (1024, 512, 96, 96, 64)])
def test_forward_lds_staged_q_o_bitwise(fa, N, Nk, d, dv, B):
    """The default geometries stage Q (LDS-DMA) and O (16-B row stores) through an
    LDS image when N % 8 == 0: bitwise equal to the per-element gathers / stores
    (variant 20), partial last query block included.  Grids of >= 256 workgroups
    (or one key tile), so neither run takes the split-KV path."""
    L = fa.lib()
    rng = np.random.default_rng(N + Nk * 3 + d)
    Q, K, V = (fa.jl_tensor(rng.standard_normal(sh), torch.bfloat16) for sh in ((N, d, B), (Nk, d, B), (Nk, dv, B)))
    a = [t.clone() for t in fa.dense_fa(Q, K, V)]
    old = L.fa_debug_set_fwd_variant(20)
    try:
        b = fa.dense_fa(Q, K, V)
        torch.cuda.synchronize()
    finally:
        L.fa_debug_set_fwd_variant(old)
    for x, y, nm in zip(a, b, ("y", "l", "m")):
        assert torch.equal(x, y), nm


def test_empty_inputs(fa):
    """Empty arrays as dense_fa! treats them (src/dense.jl:21-102): N = 0 or batch = 0
    runs no tile; Nk = 0 leaves the initial O = 0, l = 0, m = -Inf (:58-60).  The
    backward's sums over an empty key or query range are 0."""
    dev = "cuda"
    for N, Nk, B in ((0, 10, 2), (7, 10, 0)):
        q = fa.jl_empty((N, 64, B), torch.bfloat16, dev)
        k = fa.jl_empty((Nk, 64, B), torch.bfloat16, dev); k.copy_(torch.randn(k.shape))
        v = fa.jl_empty((Nk, 32, B), torch.bfloat16, dev); v.copy_(torch.randn(v.shape))
        y, l, m = fa.dense_fa(q, k, v)
        torch.cuda.synchronize()
        assert tuple(y.shape) == (N, 32, B) and tuple(l.shape) == (N, 1, B)
    q = fa.jl_empty((5, 64, 2), torch.bfloat16, dev); q.copy_(torch.randn(q.shape))
    k = fa.jl_empty((0, 64, 2), torch.bfloat16, dev)
    v = fa.jl_empty((0, 32, 2), torch.bfloat16, dev)
    y, l, m = fa.dense_fa(q, k, v)
    torch.cuda.synchronize()
    assert tuple(y.shape) == (5, 32, 2)
    assert bool((y.float() == 0).all()) and bool((l == 0).all()) and bool(torch.isneginf(m).all())
    dO = fa.jl_empty((5, 32, 2), torch.bfloat16, dev); dO.copy_(torch.randn(dO.shape))
    dq, dk, dv = fa.dense_fa_backward(q, k, v, y, dO, l, m)
    torch.cuda.synchronize()
    assert tuple(dq.shape) == (5, 64, 2) and bool((dq.float() == 0).all())
    assert tuple(dk.shape) == (0, 64, 2) and tuple(dv.shape) == (0, 32, 2)


def test_empty_batch_other_entries(fa):
    """An empty batch through windowed_fa / its backward / window / unwindow,
    circulant_fa (also N = 0) and fused_softmax: the reference loops over zero
    images, rows or slabs (src/windowed.jl:3-23, src/circulant.jl:19-46,
    src/fused_softmax.jl:1-41), so each returns correctly shaped empty outputs."""
    dev = "cuda"
    q = fa.jl_empty((16, 16, 8, 0), torch.bfloat16, dev)
    y, l, m = fa.windowed_fa(q, q, q, 7)
    torch.cuda.synchronize()
    assert tuple(y.shape) == (16, 16, 8, 0) and tuple(l.shape) == (49, 1, 9, 0)
    dq, dk, dv = fa.windowed_fa_backward(q, q, q, y, y, l, m, 7)
    torch.cuda.synchronize()
    assert tuple(dq.shape) == (16, 16, 8, 0) and tuple(dv.shape) == (16, 16, 8, 0)
    X = fa.window(q, 7)
    assert tuple(X.shape) == (49, 8, 9, 0)
    x = fa.unwindow(X, (16, 16, 8, 0), 7)
    torch.cuda.synchronize()
    assert tuple(x.shape) == (16, 16, 8, 0)
    for N, B in ((0, 2), (64, 0)):
        Q = fa.jl_empty((N, 32, B), torch.bfloat16, dev)
        O, lc, mc = fa.circulant_fa(Q, Q, Q, 5)
        torch.cuda.synchronize()
        assert tuple(O.shape) == (N, 32, B) and tuple(lc.shape) == (N, 1, B)
    S = fa.jl_empty((8, 8, 0), torch.float32, dev)
    P = fa.fused_softmax(S, dims=1)
    torch.cuda.synchronize()
    assert tuple(P.shape) == (8, 8, 0)


# Tight error budget for the 16-bit forward, beyond the generic 2e-2·(1+|y|)
# envelope of conftest.TOL: the output is rounded to T once (half an ulp: 2^-9
# relative for bf16, 2^-12 for fp16) and P is quantised to T before the PV
# product (the lazy rescale lets P reach 2^8 first), so every element
# must sit within a few output ulps of the float64 oracle on the same
# T-representable inputs, and the mean error far below one ulp.
BUDGET = {"bfloat16": (4e-3, 2e-3, 1.5e-3), "float16": (1e-3, 4e-4, 2e-4)}   # rel, abs, mean rel


@pytest.mark.parametrize("dtype", ["bfloat16", "float16"])
@pytest.mark.parametrize("case", ["golden", "cfg1_slabs"])
def test_forward_16bit_error_budget(fa, dtype, case):
    rel, ab, mean = BUDGET[dtype]
    cases = []
    if case == "golden":
        for path in golden_files("dense_"):
            g = load_golden(path)
            cases.append((g["q"], g["k"], g["v"], g["y"].astype(np.float64)))
    else:   # two slabs of configs[1]'s shape, randn inputs rounded to T
        rng = np.random.default_rng(99)
        rt = lambda a: torch.tensor(a).to(DT[dtype]).double().numpy()
        q, k, v = (rt(rng.standard_normal((4096, 64, 2))) for _ in range(3))
        cases.append((q, k, v, O.dense_fa3(q, k, v)[0]))
    worst = worst_mean = 0.0
    for q, k, v, yr in cases:
        y, _, _ = fa.dense_fa(*(fa.jl_tensor(a, DT[dtype]) for a in (q, k, v)))
        torch.cuda.synchronize()
        yg = _np(y).reshape(yr.shape)
        err = np.abs(yg - yr)
        ratio = (err / (rel * np.abs(yr) + ab)).max()
        worst = max(worst, ratio)
        assert ratio <= 1.0, f"{dtype}: max err {err.max():.3e} beyond {rel}·|y| + {ab} (ratio {ratio:.2f})"
        mlim = mean * np.abs(yr).mean() + ab / 20
        assert err.mean() <= mlim, f"{dtype}: mean err {err.mean():.3e} > {mlim:.3e}"
        worst_mean = max(worst_mean, err.mean() / mlim)
    print(f"{dtype} {case}: worst max err / budget = {worst:.3f}, worst mean err / budget = {worst_mean:.3f}")
