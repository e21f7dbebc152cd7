"""CPU oracle for the dense / windowed flash-attention hot path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module, and only as the
checker.  The product path (``flashattention.jl_amd``) never imports it and has
no CPU fallback.

This is a numpy float64 restatement of the reference algorithms of
nikopj/FlashAttention.jl (read-only at /root/reference).  Every function cites
the reference file:line it follows.  Arrays use the reference's Julia shapes
(``(spatial..., d, batch)``; the memory order of the numpy array is irrelevant
here, numpy indexes by shape).

Parity pinning — "parity unpinned" by reference-executed vectors
-------------------------------------------------------------------
The reference is Julia and cannot run here (no Julia, no NNlib), its C++
counterpart needs Eigen3 (absent: unbuildable), and it ships no golden
vectors or known-answer tests.  So no value in
tests/golden/ was produced by the reference itself: parity is UNPINNED in
that strict sense.  What this restatement IS checked against
(tests/test_oracle.py):
  * the reference's own test relations — dense_fa ≈ dense_dpa ≈
    NNlib.dot_product_attention (test/test.jl:19-20, bench/compare.jl:20,47),
    with torch CPU ``scaled_dot_product_attention`` standing in for NNlib;
  * the backward against torch autograd (the reference has no backward test);
  * window geometry against torch ``F.unfold`` / ``F.fold`` (NNlib im2col /
    col2im with cross-correlation order, ``flipped=true``; the NNlib version is
    unpinned: no ``[compat]`` in Project.toml:6-19, Manifest gitignored).
"""
from __future__ import annotations

import math
from typing import Sequence, Tuple

import numpy as np

CACHE_M = 32_000  # "≈ cache size" constant, src/dense.jl:28 and :113


def _cld(a: int, b: int) -> int:
    return -(-a // b)


def tile_policy(N: int, d: int, M: int = CACHE_M) -> Tuple[int, int]:
    """Row / column block lengths of ``dense_fa!``.

    src/dense.jl:34-35: ``Bc = clamp(cld(M, d), 1, N)``,
    ``Br = clamp(min(d, cld(M, d)), 1, N)``.
    """
    Bc = min(max(_cld(M, d), 1), N)
    Br = min(max(min(d, _cld(M, d)), 1), N)
    return Br, Bc


# --------------------------------------------------------------------------
# naive oracle: dense_dpa
# --------------------------------------------------------------------------
def dense_dpa3(Q: np.ndarray, K: np.ndarray, V: np.ndarray):
    """``dense_dpa!(O, P, Q, K, V)`` — src/naive/dense.jl:8-18.

    P = softmax_rows(Q Kᵀ / √d) (:14-15, NNlib.softmax! dims=2), O = P V (:16).
    Q, K: (N, d, B); V: (Nk, dv, B).  Returns O (N, dv, B), P (N, Nk, B).
    """
    Q = np.asarray(Q, dtype=np.float64)
    K = np.asarray(K, dtype=np.float64)
    V = np.asarray(V, dtype=np.float64)
    d = Q.shape[1]
    S = np.einsum("nkb,jkb->njb", Q, K) * (1.0 / math.sqrt(d))
    S = S - S.max(axis=1, keepdims=True)
    P = np.exp(S)
    P /= P.sum(axis=1, keepdims=True)
    O = np.einsum("njb,jcb->ncb", P, V)
    return O, P


def dense_dpa(q, k, v):
    """N-D wrapper ``dense_dpa(q, k, v)`` — src/naive/dense.jl:20-35."""
    q = np.asarray(q)
    D = q.ndim
    dqk, bs = q.shape[D - 2], q.shape[D - 1]
    dvo = v.shape[D - 2]
    Q = np.reshape(q, (-1, dqk, bs), order="F")
    K = np.reshape(k, (-1, dqk, bs), order="F")
    V = np.reshape(v, (-1, dvo, bs), order="F")
    O, P = dense_dpa3(Q, K, V)
    y = np.reshape(O, q.shape[: D - 2] + (dvo, bs), order="F")
    return y, P


# --------------------------------------------------------------------------
# blockwise FA-1 forward: dense_fa!
# --------------------------------------------------------------------------
def dense_fa3(Q, K, V, M: int = CACHE_M):
    """Blockwise forward ``dense_fa!(O, l, m, Q, K, V)`` — src/dense.jl:21-102.

    Same tile policy (:28-41), same per-tile FA-1 update with O kept normalised
    every step (:77-91).  Returns O (N, dv, B), l (N, 1, B), m (N, 1, B) with
    l = Σⱼ exp(sᵢⱼ − mᵢ), m = maxⱼ sᵢⱼ, s = τ Q Kᵀ, τ = 1/√d (:43).

    Generalisations (documented deviations): Nk may differ from N
    (the reference indexes K with N, :46-71), and dv may differ from d (the
    reference allocates O with d columns, :11/:62, Appendix A.1).
    """
    Q = np.asarray(Q, dtype=np.float64)
    K = np.asarray(K, dtype=np.float64)
    V = np.asarray(V, dtype=np.float64)
    N, d, B = Q.shape
    Nk = K.shape[0]
    dv = V.shape[1]
    Br, _ = tile_policy(N, d, M)
    _, Bc = tile_policy(Nk, d, M)
    tau = 1.0 / math.sqrt(d)
    O = np.zeros((N, dv, B))
    l = np.zeros((N, 1, B))
    m = np.full((N, 1, B), -np.inf)
    Tr, Tc = _cld(N, Br), _cld(Nk, Bc)
    for i in range(Tr):                      # @threads over (b, i), :45
        r0, r1 = i * Br, min(N, (i + 1) * Br)
        Qi = Q[r0:r1]
        Oi = np.zeros((r1 - r0, dv, B))      # fill!(Oi, 0)   :58
        li = np.zeros((r1 - r0, B))          # fill!(li, 0)   :59
        mi = np.full((r1 - r0, B), -np.inf)  # fill!(mi, -Inf) :60
        for j in range(Tc):                  # :70
            c0, c1 = j * Bc, min(Nk, (j + 1) * Bc)
            Kj, Vj = K[c0:c1], V[c0:c1]
            Pij = np.einsum("nkb,jkb->njb", Qi, Kj) * tau   # :77
            mij = Pij.max(axis=1)                            # :78
            Pij = np.exp(Pij - mij[:, None, :])              # :79
            lij = Pij.sum(axis=1)                            # :80
            mi_new = np.maximum(mi, mij)                     # :82
            ei = np.exp(mi - mi_new)                         # :83
            eij = np.exp(mij - mi_new)                       # :84
            li_new = ei * li + eij * lij                     # :85
            Oi_new = np.einsum("njb,jcb->ncb", Pij, Vj)      # :88
            Oi = ((li * ei)[:, None, :] * Oi + eij[:, None, :] * Oi_new) / li_new[:, None, :]  # :89
            li, mi = li_new, mi_new                          # :90-91
        O[r0:r1] = Oi
        l[r0:r1, 0] = li
        m[r0:r1, 0] = mi
    return O, l, m


def dense_fa(q, k, v, M: int = CACHE_M):
    """N-D wrapper ``dense_fa(q, k, v) -> (y, l, m)`` — src/dense.jl:1-19.

    Spatial dims are flattened (column-major) into N (:6-8); y has v's feature
    count dv (the reference's ``similar(Q)`` bug, Appendix A.1, is not
    inherited).
    """
    q = np.asarray(q)
    D = q.ndim
    d, bs = q.shape[D - 2], q.shape[D - 1]
    dv = v.shape[D - 2]
    Q = np.reshape(q, (-1, d, bs), order="F")
    K = np.reshape(k, (-1, d, bs), order="F")
    V = np.reshape(v, (-1, dv, bs), order="F")
    O, l, m = dense_fa3(Q, K, V, M)
    y = np.reshape(O, q.shape[: D - 2] + (dv, bs), order="F")
    return y, l, m


# --------------------------------------------------------------------------
# backward
# --------------------------------------------------------------------------
def dense_fa_backward(Q, K, V, O, dO, l, m, M: int = CACHE_M):
    """Blockwise backward — executable spec ``OneDFastBack``
    src_cpp/FlashAttention.cpp:194-252 (loop :221-251, math :238-246), with
    λ = τ = 1/√d as in the Julia intent src/dense.jl:131-162.

    P = exp(τ Q Kᵀ − m)/l (:237-238); dV += Pᵀ dO (:239); dP = dO Vᵀ (:240);
    D = rowsum(dO∘O) (:241); dS = P∘(dP − D) (:242); dQ += τ dS K (:243);
    dK += τ dSᵀ Q (:244).  dQ, dK, dV start at zero (the Julia ``similar``
    + ``+=`` bug, Appendix A.2, is not inherited).

    Shapes: Q (N, d, B); K (Nk, d, B); V (Nk, dv, B); O, dO (N, dv, B);
    l, m (N, 1, B) or (N, B).  Returns dQ (N, d, B), dK (Nk, d, B),
    dV (Nk, dv, B).
    """
    Q = np.asarray(Q, dtype=np.float64)
    K = np.asarray(K, dtype=np.float64)
    V = np.asarray(V, dtype=np.float64)
    O = np.asarray(O, dtype=np.float64)
    dO = np.asarray(dO, dtype=np.float64)
    N, d, B = Q.shape
    Nk = K.shape[0]
    l = np.asarray(l, dtype=np.float64).reshape(N, B)
    m = np.asarray(m, dtype=np.float64).reshape(N, B)
    tau = 1.0 / math.sqrt(d)
    Br, _ = tile_policy(N, d, M)
    _, Bc = tile_policy(Nk, d, M)
    dQ = np.zeros_like(Q)
    dK = np.zeros_like(K)
    dV = np.zeros_like(V)
    for i in range(_cld(N, Br)):
        r0, r1 = i * Br, min(N, (i + 1) * Br)
        Qi, Oi, dOi = Q[r0:r1], O[r0:r1], dO[r0:r1]
        li, mi = l[r0:r1], m[r0:r1]
        Di = np.sum(dOi * Oi, axis=1)                               # :241
        for j in range(_cld(Nk, Bc)):
            c0, c1 = j * Bc, min(Nk, (j + 1) * Bc)
            Kj, Vj = K[c0:c1], V[c0:c1]
            S = np.einsum("nkb,jkb->njb", Qi, Kj) * tau             # :236
            P = np.exp(S - mi[:, None, :]) / li[:, None, :]         # :237-238
            dV[c0:c1] += np.einsum("njb,ncb->jcb", P, dOi)          # :239
            dP = np.einsum("ncb,jcb->njb", dOi, Vj)                 # :240
            dS = P * (dP - Di[:, None, :])                          # :242
            dQ[r0:r1] += tau * np.einsum("njb,jkb->nkb", dS, Kj)    # :243
            dK[c0:c1] += tau * np.einsum("njb,nkb->jkb", dS, Qi)    # :244
    return dQ, dK, dV


# --------------------------------------------------------------------------
# window / unwindow (NNlib unfold / fold semantics)
# --------------------------------------------------------------------------
def window_geometry(spatial: Sequence[int], ws: int, stride: int, pad: int):
    """Output grid of ``NNlib.unfold(x, (ws…, d, 1); stride, pad)``
    (src/utils.jl:40): per spatial dim ⌊(Sᵢ + 2p − ws)/s⌋ + 1 windows."""
    out = tuple((s + 2 * pad - ws) // stride + 1 for s in spatial)
    if any(o <= 0 for o in out):
        raise ValueError("window larger than padded input")
    return out


def window_index(spatial: Sequence[int], ws: int, stride: int, pad: int) -> np.ndarray:
    """Gather index ``idx[t, w]`` into the column-major flattened spatial grid,
    −1 where the window reads zero padding.

    t = window-local token (first spatial dim fastest, src/utils.jl:41-42 with
    NNlib im2col cross-correlation order); w = window index (first output dim
    fastest).
    """
    k = len(spatial)
    out = window_geometry(spatial, ws, stride, pad)
    # window-local offsets, first dim fastest
    offs = np.stack(np.meshgrid(*[np.arange(ws)] * k, indexing="ij"), -1)
    offs = offs.transpose(*reversed(range(k)), k).reshape(-1, k)       # (ws^k, k)
    wins = np.stack(np.meshgrid(*[np.arange(o) for o in out], indexing="ij"), -1)
    wins = wins.transpose(*reversed(range(k)), k).reshape(-1, k)       # (L, k)
    coord = wins[None, :, :] * stride - pad + offs[:, None, :]         # (ws^k, L, k)
    valid = np.all((coord >= 0) & (coord < np.asarray(spatial)), axis=-1)
    strides = np.cumprod((1,) + tuple(spatial[:-1]))
    flat = np.sum(coord * strides, axis=-1)
    return np.where(valid, flat, -1)


def window(x, ws: int, stride: int | None = None, pad: int | None = None):
    """``window(x, ws; stride=ws, pad=(ws-1)÷2)`` — src/utils.jl:36-44.

    (spatial..., d, B) → (ws^k, d, L, B)."""
    stride = ws if stride is None else stride
    pad = (ws - 1) // 2 if pad is None else pad
    x = np.asarray(x, dtype=np.float64)
    spatial, d, B = x.shape[:-2], x.shape[-2], x.shape[-1]
    idx = window_index(spatial, ws, stride, pad)
    xf = np.reshape(x, (-1, d, B), order="F")
    X = np.where((idx >= 0)[:, :, None, None], xf[np.maximum(idx, 0)], 0.0)  # (T, L, d, B)
    return X.transpose(0, 2, 1, 3).copy()                                    # (T, d, L, B)


def unwindow(X, outsize: Sequence[int], ws: int, stride: int | None = None,
             pad: int | None = None):
    """``unwindow(X, outsize, ws; stride, pad)`` — src/utils.jl:46-54
    (NNlib.fold: overlapping contributions are SUMMED, padding dropped).

    (ws^k, d, L, B) → outsize = (spatial..., d, B)."""
    stride = ws if stride is None else stride
    pad = (ws - 1) // 2 if pad is None else pad
    X = np.asarray(X, dtype=np.float64)
    spatial, d, B = tuple(outsize[:-2]), outsize[-2], outsize[-1]
    idx = window_index(spatial, ws, stride, pad)                      # (T, L)
    n = int(np.prod(spatial))
    acc = np.zeros((n + 1, d, B))
    tgt = np.where(idx >= 0, idx, n)                                  # pad → dump row
    np.add.at(acc, tgt.reshape(-1), X.transpose(0, 2, 1, 3).reshape(-1, d, B))
    return np.reshape(acc[:n], tuple(spatial) + (d, B), order="F")


def coverage(spatial: Sequence[int], ws: int, stride: int, pad: int) -> np.ndarray:
    """Per-pixel window count (the ``divisor`` of src/windowed.jl:16-17)."""
    idx = window_index(spatial, ws, stride, pad)
    n = int(np.prod(spatial))
    cnt = np.bincount(idx[idx >= 0].reshape(-1), minlength=n).astype(np.float64)
    return np.reshape(cnt, tuple(spatial), order="F")


def windowed_fa(q, k, v, ws: int, stride: int | None = None, pad: int | None = None,
                attn=None):
    """``windowed_fa(q, k, v, ws; stride=ws, pad=(ws-1)÷2)`` — src/windowed.jl:3-23.

    window q, k, v (:4-6) → dense_fa on (ws^k, d, L·B) (:8-11) → fold ÷
    coverage count (:16-19).  Pixels no window covers come out 0/0 = NaN
    (Appendix A.7; reproduced, not fixed).  Returns y (spatial..., dv, B),
    l, m (ws^k, 1, L, B) in window layout (:20-21).
    """
    stride = ws if stride is None else stride
    pad = (ws - 1) // 2 if pad is None else pad
    q = np.asarray(q, dtype=np.float64)
    qw = window(q, ws, stride, pad)
    kw = window(k, ws, stride, pad)
    vw = window(v, ws, stride, pad)
    T, d, L, B = qw.shape
    dv = vw.shape[1]
    r = lambda a: np.reshape(a, (a.shape[0], a.shape[1], -1), order="F")
    if attn is None:
        yw, lw, mw = dense_fa3(r(qw), r(kw), r(vw))
    else:
        yw, lw, mw = attn(r(qw), r(kw), r(vw))
    yw = np.reshape(yw, (T, dv, L, B), order="F")
    szy = tuple(q.shape[:-2]) + (dv, q.shape[-1])
    with np.errstate(invalid="ignore", divide="ignore"):
        div = coverage(q.shape[:-2], ws, stride, pad)
        y = unwindow(yw, szy, ws, stride, pad) / div.reshape(div.shape + (1, 1))
    lw = np.reshape(lw, (T, 1, L, B), order="F")
    mw = np.reshape(mw, (T, 1, L, B), order="F")
    return y, lw, mw


def block_fa(q, k, v, ws: int, pad: int = 0):
    """``block_fa`` = windowed_fa with stride = ws — src/windowed.jl:1."""
    return windowed_fa(q, k, v, ws, stride=ws, pad=pad)


def windowed_dpa(q, k, v, ws: int, stride: int | None = None, pad: int | None = None):
    """``windowed_dpa`` — src/naive/windowed.jl:3-22 (returns y only here)."""
    def attn(Q, K, V):
        O, _ = dense_dpa3(Q, K, V)
        return O, None, None
    stride = ws if stride is None else stride
    pad = (ws - 1) // 2 if pad is None else pad
    q = np.asarray(q, dtype=np.float64)
    qw, kw, vw = (window(a, ws, stride, pad) for a in (q, k, v))
    T, d, L, B = qw.shape
    dv = vw.shape[1]
    r = lambda a: np.reshape(a, (a.shape[0], a.shape[1], -1), order="F")
    yw, _ = dense_dpa3(r(qw), r(kw), r(vw))
    yw = np.reshape(yw, (T, dv, L, B), order="F")
    szy = tuple(q.shape[:-2]) + (dv, q.shape[-1])
    with np.errstate(invalid="ignore", divide="ignore"):
        div = coverage(q.shape[:-2], ws, stride, pad)
        return unwindow(yw, szy, ws, stride, pad) / div.reshape(div.shape + (1, 1))


def windowed_fa_backward(q, k, v, dy, ws: int, stride: int | None = None,
                         pad: int | None = None):
    """Composed windowed backward (the reference README
    claims it, README.md:36-37, no code exists): dyw = window(dy ./ divisor),
    dense backward per window, fold(dqw/dkw/dvw).  Chain rule of
    ``windowed_fa`` exactly (window/unwindow are adjoint linear maps)."""
    stride = ws if stride is None else stride
    pad = (ws - 1) // 2 if pad is None else pad
    q = np.asarray(q, dtype=np.float64)
    k = np.asarray(k, dtype=np.float64)
    v = np.asarray(v, dtype=np.float64)
    qw, kw, vw = (window(a, ws, stride, pad) for a in (q, k, v))
    T, d, L, B = qw.shape
    dv = vw.shape[1]
    r = lambda a: np.reshape(a, (a.shape[0], a.shape[1], -1), order="F")
    Ow, lw, mw = dense_fa3(r(qw), r(kw), r(vw))
    div = coverage(q.shape[:-2], ws, stride, pad)
    with np.errstate(invalid="ignore", divide="ignore"):
        g = np.asarray(dy, dtype=np.float64) / div.reshape(div.shape + (1, 1))
    dyw = window(g, ws, stride, pad)
    dQw, dKw, dVw = dense_fa_backward(r(qw), r(kw), r(vw), Ow, r(dyw), lw, mw)
    sp = tuple(q.shape[:-2])
    dq = unwindow(np.reshape(dQw, (T, d, L, B), order="F"), sp + (d, q.shape[-1]), ws, stride, pad)
    dk = unwindow(np.reshape(dKw, (T, d, L, B), order="F"), sp + (d, q.shape[-1]), ws, stride, pad)
    dvv = unwindow(np.reshape(dVw, (T, dv, L, B), order="F"), sp + (dv, q.shape[-1]), ws, stride, pad)
    return dq, dk, dvv


# ---------------------------------------------------------------------------
# circulant (periodic banded) attention — SURVEY §8f row 3
# ---------------------------------------------------------------------------
def circshift_index(m: int, s: int, M: int) -> int:
    """``circshift_index(m, s, M)`` — src/utils.jl:4 (1-based)."""
    return (m - 1 - s) % M + 1


def cartesian_circulant(n: int, N: int, M: int) -> Tuple[int, int]:
    """``cartesian_circulant(n, N, M)`` — src/utils.jl:6-17 (1-based (i, j)):
    entry n of the column-major N×N circulant with M nonzeros per column."""
    p = (M - 1) // 2
    j = _cld(n, M)
    m = (n - 1) % M + 1
    if j <= p:
        m = circshift_index(m, j - p - 1, M)
    elif j > N - p:
        m = circshift_index(m, p - N + j, M)
    i = ((m - 1) + (j - 1) - p) % N + 1
    return i, j


def circulant_index(N: int, W: int) -> np.ndarray:
    """0-based key index ``J[w, i]`` of band entry w of query i, exactly as the
    reference loops compute it: ``jjj = cartesian_circulant((i-1)*W + w, N, W)[1]``
    (src/circulant.jl:74-75, src/naive/circulant.jl:21-22)."""
    J = np.empty((W, N), dtype=np.int64)
    for i in range(N):
        for w in range(W):
            J[w, i] = cartesian_circulant(i * W + w + 1, N, W)[0] - 1
    return J


def circulant_dpa3(Q, K, V, W: int):
    """``circulant_dpa!(O, P, Q, K, V, W)`` — src/naive/circulant.jl:8-36:
    band scores P[w, i] = τ qᵢ·k_J[w,i], softmax over w (dims=1), O = Pᵀ-circulant · V.
    Returns O (N, dv, B) and P (W, N, B)."""
    Q = np.asarray(Q, dtype=np.float64)
    K = np.asarray(K, dtype=np.float64)
    V = np.asarray(V, dtype=np.float64)
    N, d, B = Q.shape
    dv = V.shape[1]
    tau = 1.0 / math.sqrt(d)
    J = circulant_index(N, W)
    O = np.zeros((N, dv, B))
    P = np.zeros((W, N, B))
    for b in range(B):
        S = tau * np.einsum("nk,wnk->wn", Q[:, :, b], K[J, :, b])   # :19-24
        S = np.exp(S - S.max(axis=0, keepdims=True))
        S /= S.sum(axis=0, keepdims=True)                             # softmax!(P, dims=1), :27
        P[:, :, b] = S
        O[:, :, b] = np.einsum("wn,wnc->nc", S, V[J, :, b])          # P * bV, :28-34
    return O, P


def circulant_fa3(Q, K, V, W: int, M: int = CACHE_M):
    """Blockwise ``circulant_fa!(O, l, m, Q, K, V, W)`` — src/circulant.jl:9-118.

    Tile policy Bw = clamp(cld(M, d), 1, W), Br = clamp(min(d, cld(M, d)), 1, N)
    (:22-25); per (row block, window block) the FA-1 update of dense_fa! (:80-103)
    with O kept normalised.  Returns O (N, dv, B), l, m (N, 1, B).  dv may differ
    from d (the reference allocates O like Q, :3).
    """
    Q = np.asarray(Q, dtype=np.float64)
    K = np.asarray(K, dtype=np.float64)
    V = np.asarray(V, dtype=np.float64)
    N, d, B = Q.shape
    dv = V.shape[1]
    Bw = min(max(_cld(M, d), 1), W)
    Br = min(max(min(d, _cld(M, d)), 1), N)
    tau = 1.0 / math.sqrt(d)
    J = circulant_index(N, W)
    O = np.zeros((N, dv, B))
    l = np.zeros((N, 1, B))
    m = np.full((N, 1, B), -np.inf)
    for i in range(_cld(N, Br)):
        r0, r1 = i * Br, min(N, (i + 1) * Br)
        Oi = np.zeros((r1 - r0, dv, B))
        li = np.zeros((r1 - r0, B))
        mi = np.full((r1 - r0, B), -np.inf)
        for w in range(_cld(W, Bw)):
            w0, w1 = w * Bw, min(W, (w + 1) * Bw)
            Jw = J[w0:w1, r0:r1]                                          # (nw, nr)
            Piw = tau * np.einsum("nkb,wnkb->nwb", Q[r0:r1], K[Jw])       # :70-79
            miw = Piw.max(axis=1)                                         # :80
            Piw = np.exp(Piw - miw[:, None, :])                           # :81
            liw = Piw.sum(axis=1)                                         # :82
            mi_new = np.maximum(mi, miw)                                  # :84
            ei = np.exp(mi - mi_new)                                      # :85
            eiw = np.exp(miw - mi_new)                                    # :86
            li_new = ei * li + eiw * liw                                  # :87
            t = np.einsum("nwb,wncb->ncb", Piw, V[Jw])                    # :90-100
            Oi = ((li * ei)[:, None, :] * Oi + eiw[:, None, :] * t) / li_new[:, None, :]   # :101
            li, mi = li_new, mi_new                                       # :106-107
        O[r0:r1] = Oi
        l[r0:r1, 0] = li
        m[r0:r1, 0] = mi
    return O, l, m


# ---------------------------------------------------------------------------
# standalone fused softmax — SURVEY §8f row 4
# ---------------------------------------------------------------------------
def fused_softmax(S, dims: int = 1):
    """``fused_softmax(S; dims)`` — src/fused_softmax.jl:1-41: vector, matrix or
    3-array; dims = 1 → ``col_softmax!`` (:30-41, each S[:, j, b]), dims = 2 →
    ``row_softmax!`` (:17-28, each S[i, :, b]).  Per vector: s .- maximum(s),
    exp, ./ sum (so an all -Inf vector, or one holding NaN / +Inf, is NaN)."""
    assert dims in (1, 2), "only softmax in dims 1 or 2 supported"   # :12
    S = np.asarray(S, dtype=np.float64)
    ax = dims - 1
    with np.errstate(invalid="ignore", over="ignore"):
        num = np.exp(S - S.max(axis=ax, keepdims=True))
        return num / num.sum(axis=ax, keepdims=True)
