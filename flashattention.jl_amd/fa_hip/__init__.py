"""fa_hip — Python host mirror of FlashAttention.jl's attention API over the
MI355X C ABI (``include/fa_hip.h``, ``libfa_hip.so``).

The reference API is Julia (nikopj/FlashAttention.jl); this module mirrors it
name for name so the parity tests read like the reference's own tests:

=========================================  ===========================================
reference (Julia)                          here (torch tensors on a ROCm device)
=========================================  ===========================================
``dense_fa(q, k, v) -> (y, l, m)``         :func:`dense_fa`        src/dense.jl:1-19
``dense_fa!(O, l, m, Q, K, V)``            :func:`dense_fa_`       src/dense.jl:21-102
``dense_fa_backward(Q,K,V,O,dO,l,m)``      :func:`dense_fa_backward` src/dense.jl:104-167
``windowed_fa(q,k,v,ws; stride, pad)``     :func:`windowed_fa`     src/windowed.jl:3-23
``block_fa(q,k,v,ws; pad=0)``              :func:`block_fa`        src/windowed.jl:1
=========================================  ===========================================

Arrays carry the reference's **Julia shapes and column-major layout**: a Julia
``(N, d, B)`` array is a torch tensor of shape ``(N, d, B)`` with strides
``(1, N, N*d)`` (create them with :func:`jl_empty` / :func:`jl_tensor`).  The
C ABI receives the raw device pointers, so no copy or transpose happens at the
boundary.  ``l`` and ``m`` are float32 for every input dtype.

Errors mirror the reference: shape problems raise :class:`DimensionMismatch`
(Julia ``DimensionMismatch``); failures reported by the library raise
:class:`FlashAttentionError` carrying ``fa_last_error()``.  There is no CPU
fallback: if ``libfa_hip.so`` is missing, importing the bindings fails loudly.
"""
from __future__ import annotations

import ctypes
import math
import os
from typing import Optional, Sequence, Tuple

import torch

__all__ = [
    "DimensionMismatch", "FlashAttentionError", "lib", "lib_path",
    "jl_empty", "jl_zeros", "jl_tensor", "jl_strides", "is_jl_contiguous",
    "dense_fa", "dense_fa_", "dense_fa_backward", "backward_handoff_status", "backward_handoff_trips",
    "windowed_fa", "block_fa",
    "windowed_fa_backward", "window_geometry", "circulant_fa", "circulant_fa_", "circulant_dpa",
    "fused_softmax", "fused_softmax_", "DTYPES",
]

_HERE = os.path.dirname(os.path.abspath(__file__))
_PKG = os.path.dirname(_HERE)


class DimensionMismatch(ValueError):
    """Raised where the reference's Julia code throws ``DimensionMismatch``."""


class FlashAttentionError(RuntimeError):
    """A nonzero ``fa_status`` from the C ABI; message = ``fa_last_error()``."""

    def __init__(self, status: int, message: str):
        super().__init__(f"[fa_status {status}] {message}")
        self.status = status


FA_OK, FA_ERR_INVALID_ARG, FA_ERR_UNSUPPORTED, FA_ERR_HIP, FA_ERR_WORKSPACE = range(5)
DTYPES = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2, torch.float64: 3}

# ----------------------------------------------------------------------------
# library loading (the C ABI is the only compute path)
# ----------------------------------------------------------------------------
_LIB = None


def lib_path() -> str:
    return os.environ.get("FA_HIP_LIB", os.path.join(_PKG, "libfa_hip.so"))


def lib() -> ctypes.CDLL:
    """Load ``libfa_hip.so`` (built by ``__graft_entry__.build()``).

    torch is imported first so the library binds torch's already-loaded HIP
    runtime (same soname), i.e. device pointers and streams are shared.
    """
    global _LIB
    if _LIB is not None:
        return _LIB
    path = lib_path()
    if not os.path.exists(path):
        raise ImportError(
            f"fa_hip: native library not found at {path}; run __graft_entry__.build() "
            "(there is deliberately no CPU fallback)")
    L = ctypes.CDLL(path)
    i64, f32, vp = ctypes.c_int64, ctypes.c_float, ctypes.c_void_p
    fp = ctypes.POINTER(ctypes.c_float)
    L.fa_last_error.restype = ctypes.c_char_p
    L.fa_abi_version.restype = ctypes.c_int
    L.fa_max_head_dim.restype = ctypes.c_int
    L.fa_dense_fwd.restype = ctypes.c_int
    L.fa_dense_fwd.argtypes = [ctypes.c_int, vp, vp, vp, vp, vp, vp, i64, i64, i64, i64, i64, f32, vp]
    L.fa_dense_bwd_workspace.restype = ctypes.c_size_t
    L.fa_dense_bwd_workspace.argtypes = [ctypes.c_int, i64, i64, i64, i64, i64]
    L.fa_dense_bwd.restype = ctypes.c_int
    L.fa_dense_bwd.argtypes = [ctypes.c_int, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp,
                               i64, i64, i64, i64, i64, f32, vp, ctypes.c_size_t, vp]
    L.fa_dense_bwd_handoff_status.restype = ctypes.c_int
    L.fa_dense_bwd_handoff_status.argtypes = [vp, ctypes.c_size_t, vp, ctypes.POINTER(ctypes.c_int)]
    L.fa_windowed_workspace.restype = ctypes.c_size_t
    L.fa_windowed_workspace.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(i64),
                                        i64, i64, i64, i64, i64, i64]
    L.fa_windowed_fwd_workspace.restype = ctypes.c_size_t
    L.fa_windowed_fwd_workspace.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(i64),
                                            i64, i64, i64, i64, i64, i64]
    L.fa_windowed_fwd.restype = ctypes.c_int
    L.fa_windowed_fwd.argtypes = [ctypes.c_int, vp, vp, vp, vp, vp, vp, ctypes.c_int,
                                  ctypes.POINTER(i64), i64, i64, i64, i64, i64, i64, f32, vp,
                                  ctypes.c_size_t, vp]
    L.fa_windowed_bwd.restype = ctypes.c_int
    L.fa_windowed_bwd.argtypes = [ctypes.c_int, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp,
                                  ctypes.c_int, ctypes.POINTER(i64), i64, i64, i64, i64, i64, i64,
                                  f32, vp, ctypes.c_size_t, vp]
    # (hasattr: tools/ab_lib.py also loads older builds for A/B timing)
    for wfn in ("fa_window", "fa_unwindow"):
        if hasattr(L, wfn):
            getattr(L, wfn).restype = ctypes.c_int
            getattr(L, wfn).argtypes = [ctypes.c_int, vp, vp, ctypes.c_int, ctypes.POINTER(i64), i64, i64,
                                        i64, i64, i64, vp]
    if hasattr(L, "fa_dense_fwd_ws"):
        L.fa_dense_fwd_ws.restype = ctypes.c_int
        L.fa_dense_fwd_ws.argtypes = [ctypes.c_int, vp, vp, vp, vp, vp, vp, i64, i64, i64, i64, i64, f32, vp,
                                      ctypes.c_size_t, vp]
        L.fa_dense_fwd_workspace.restype = ctypes.c_size_t
        L.fa_dense_fwd_workspace.argtypes = [ctypes.c_int, i64, i64, i64, i64, i64]
    L.fa_circulant_fwd.restype = ctypes.c_int
    L.fa_circulant_fwd.argtypes = [ctypes.c_int, vp, vp, vp, vp, vp, vp, i64, i64, i64, i64, i64, f32, vp]
    L.fa_softmax_workspace.restype = ctypes.c_size_t
    L.fa_softmax_workspace.argtypes = [i64, i64, i64, ctypes.c_int]
    L.fa_softmax.restype = ctypes.c_int
    L.fa_softmax.argtypes = [ctypes.c_int, vp, vp, i64, i64, i64, ctypes.c_int, vp, ctypes.c_size_t, vp]
    del fp
    for dbg in ("fa_debug_set_fwd_variant", "fa_debug_set_bwd_generic", "fa_debug_set_win_composed",
                "fa_debug_set_circ_generic", "fa_debug_set_bwd_mode"):
        if hasattr(L, dbg):
            getattr(L, dbg).restype = ctypes.c_int
            getattr(L, dbg).argtypes = [ctypes.c_int]
    if hasattr(L, "fa_debug_set_rescale_threshold"):
        L.fa_debug_set_rescale_threshold.restype = ctypes.c_float
        L.fa_debug_set_rescale_threshold.argtypes = [ctypes.c_float]
    if L.fa_abi_version() != 1:
        raise ImportError("fa_hip: ABI version mismatch")
    _LIB = L
    return L


def _check(rc: int) -> None:
    if rc != FA_OK:
        msg = lib().fa_last_error().decode(errors="replace")
        if rc == FA_ERR_INVALID_ARG and "DimensionMismatch" in msg:
            raise DimensionMismatch(msg)
        raise FlashAttentionError(rc, msg)


# ----------------------------------------------------------------------------
# Julia-layout tensors
# ----------------------------------------------------------------------------
def jl_strides(shape: Sequence[int]) -> Tuple[int, ...]:
    st, acc = [], 1
    for s in shape:
        st.append(acc)
        acc *= int(s)
    return tuple(st)


def is_jl_contiguous(t: torch.Tensor) -> bool:
    """True if ``t`` is laid out like a Julia Array of the same shape (an empty
    array trivially is: no element is ever addressed)."""
    if t.numel() == 0:
        return True
    return all(sz == 1 or st == js for sz, st, js in zip(t.shape, t.stride(), jl_strides(t.shape)))


def jl_empty(shape: Sequence[int], dtype=torch.float32, device="cuda") -> torch.Tensor:
    """Uninitialised tensor with Julia shape ``shape`` and column-major strides."""
    shape = tuple(int(s) for s in shape)
    n = len(shape)
    return torch.empty(tuple(reversed(shape)), dtype=dtype, device=device).permute(*reversed(range(n)))


def jl_zeros(shape: Sequence[int], dtype=torch.float32, device="cuda") -> torch.Tensor:
    t = jl_empty(shape, dtype, device)
    t.zero_()
    return t


def jl_tensor(x, dtype=torch.float32, device="cuda") -> torch.Tensor:
    """Copy array-like ``x`` (indexed by Julia shape) into a column-major tensor."""
    src = torch.as_tensor(x)
    t = jl_empty(src.shape, dtype, device)
    t.copy_(src)
    return t


def _ptr(t: Optional[torch.Tensor]):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def _stream(t: torch.Tensor):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def _require(cond: bool, msg: str) -> None:
    if not cond:
        raise DimensionMismatch(msg)


def _dtype_code(*ts: torch.Tensor) -> int:
    dt = ts[0].dtype
    for t in ts:
        _require(t.dtype == dt, f"mixed element types {dt} and {t.dtype}")
    if dt not in DTYPES:
        raise TypeError(f"unsupported element type {dt}; use float64, float32, bfloat16 or float16")
    return DTYPES[dt]


def _device_check(*ts: torch.Tensor) -> None:
    dev = ts[0].device
    if dev.type != "cuda":
        raise TypeError("fa_hip computes on the ROCm device only (no CPU fallback); "
                        "move arrays to 'cuda'")
    for t in ts:
        _require(t.device == dev, "arrays on different devices")
        _require(is_jl_contiguous(t), "arrays must be column-major (Julia) contiguous; "
                 "use fa_hip.jl_tensor / jl_empty")


# ----------------------------------------------------------------------------
# dense
# ----------------------------------------------------------------------------
def dense_fa_(O: torch.Tensor, l: torch.Tensor, m: torch.Tensor,
              Q: torch.Tensor, K: torch.Tensor, V: torch.Tensor,
              scale: float = 0.0) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """``dense_fa!(O, l, m, Q, K, V)`` — src/dense.jl:21-102, in place.

    Q (N, d, B), K (Nk, d, B), V (Nk, dv, B), O (N, dv, B); l, m (N, 1, B)
    float32.  Returns ``(O, l, m)`` like the reference (:101).
    """
    for t in (O, l, m, Q, K, V):
        _require(t.dim() == 3, "dense_fa! expects 3-D (N, d, batch) arrays")
    N, d, B = Q.shape
    Nk, dv = K.shape[0], V.shape[1]
    _require(K.shape == (Nk, d, B), f"K has shape {tuple(K.shape)}, expected ({Nk}, {d}, {B})")
    _require(V.shape == (Nk, dv, B), f"V has shape {tuple(V.shape)}, expected ({Nk}, {dv}, {B})")
    _require(O.shape == (N, dv, B), f"O has shape {tuple(O.shape)}, expected ({N}, {dv}, {B})")
    _require(l.shape == (N, 1, B) and m.shape == (N, 1, B), "l, m must be (N, 1, batch)")
    _require(l.dtype == torch.float32 and m.dtype == torch.float32, "l, m must be float32")
    code = _dtype_code(Q, K, V, O)
    _device_check(Q, K, V, O, l, m)
    Lb = lib()
    nws = Lb.fa_dense_fwd_workspace(code, N, Nk, d, dv, B) if hasattr(Lb, "fa_dense_fwd_ws") else 0
    if (code in (DTYPES[torch.bfloat16], DTYPES[torch.float16]) and N * Nk * B > 0 and Nk % 8 == 0
            and (K.data_ptr() % 16 or V.data_ptr() % 16)):
        # K / V not 16-B aligned (a view at an odd offset): add room for the
        # padded K / V copies the fast kernels then run on (fa_fwd.hip
        # fwd_pad_bytes_any); the shape-only workspace query cannot see pointers
        al = lambda x: (x + 255) & ~255
        nws += al(Nk * d * B * 2) + al(Nk * dv * B * 2) + 256
    if nws == 0:
        _check(Lb.fa_dense_fwd(code, _ptr(Q), _ptr(K), _ptr(V), _ptr(O), _ptr(l), _ptr(m),
                               N, Nk, d, dv, B, float(scale), _stream(Q)))
    else:   # ragged Nk: padded K / V copies let the fast kernels run
        ws = _workspace(Q.device, nws)
        _check(Lb.fa_dense_fwd_ws(code, _ptr(Q), _ptr(K), _ptr(V), _ptr(O), _ptr(l), _ptr(m),
                                  N, Nk, d, dv, B, float(scale), _ptr(ws), int(nws), _stream(Q)))
    return O, l, m


def dense_fa(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, scale: float = 0.0):
    """``dense_fa(q, k, v) -> (y, l, m)`` — src/dense.jl:1-19.

    q, k: (spatial..., d, B); v: (spatial..., dv, B).  Spatial dims are
    flattened column-major into N (:6-8).  y: (spatial..., dv, B); l, m:
    (N, 1, B) float32 with l = Σ exp(s − m), m = max s (natural-log units).
    """
    _require(q.dim() >= 3 and k.dim() == q.dim() and v.dim() == q.dim(),
             "q, k, v must share rank >= 3")
    D = q.dim()
    d, B = q.shape[D - 2], q.shape[D - 1]
    dv = v.shape[D - 2]
    _device_check(q, k, v)
    N = math.prod(q.shape[: D - 2])
    Nk = math.prod(k.shape[: D - 2])
    _require(k.shape[D - 2:] == (d, B), "k must be (spatial..., d, batch)")
    _require(math.prod(v.shape[: D - 2]) == Nk and v.shape[D - 1] == B,
             "v must have k's token count and batch")
    Q = q.as_strided((N, d, B), jl_strides((N, d, B)))
    K = k.as_strided((Nk, d, B), jl_strides((Nk, d, B)))
    V = v.as_strided((Nk, dv, B), jl_strides((Nk, dv, B)))
    O = jl_empty((N, dv, B), q.dtype, q.device)
    l = jl_empty((N, 1, B), torch.float32, q.device)
    m = jl_empty((N, 1, B), torch.float32, q.device)
    dense_fa_(O, l, m, Q, K, V, scale)
    y = O.as_strided(tuple(q.shape[: D - 2]) + (dv, B), jl_strides(tuple(q.shape[: D - 2]) + (dv, B)))
    return y, l, m


def circulant_fa_(O: torch.Tensor, l: torch.Tensor, m: torch.Tensor,
                  Q: torch.Tensor, K: torch.Tensor, V: torch.Tensor, W: int,
                  scale: float = 0.0) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """``circulant_fa!(O, l, m, Q, K, V, W)`` — src/circulant.jl:9-118, in place.

    Query i attends the W band keys (i - p + t) mod N, t = 0..W-1,
    p = (W-1)÷2 (``cartesian_circulant``, src/utils.jl:6-17).  Q, K (N, d, B),
    V (N, dv, B), O (N, dv, B), l, m (N, 1, B) float32.
    """
    for t in (O, l, m, Q, K, V):
        _require(t.dim() == 3, "circulant_fa! expects 3-D (N, d, batch) arrays")
    N, d, B = Q.shape
    dv = V.shape[1]
    _require(int(W) >= 1, "window size W must be >= 1")
    _require(K.shape == (N, d, B), f"K has shape {tuple(K.shape)}, expected ({N}, {d}, {B})")
    _require(V.shape == (N, dv, B), f"V has shape {tuple(V.shape)}, expected ({N}, {dv}, {B})")
    _require(O.shape == (N, dv, B), f"O has shape {tuple(O.shape)}, expected ({N}, {dv}, {B})")
    _require(l.shape == (N, 1, B) and m.shape == (N, 1, B), "l, m must be (N, 1, batch)")
    _require(l.dtype == torch.float32 and m.dtype == torch.float32, "l, m must be float32")
    code = _dtype_code(Q, K, V, O)
    _device_check(Q, K, V, O, l, m)
    _check(lib().fa_circulant_fwd(code, _ptr(Q), _ptr(K), _ptr(V), _ptr(O), _ptr(l), _ptr(m),
                                  N, d, dv, B, int(W), float(scale), _stream(Q)))
    return O, l, m


def circulant_fa(Q: torch.Tensor, K: torch.Tensor, V: torch.Tensor, W: int, scale: float = 0.0):
    """``circulant_fa(Q, K, V, W) -> (O, l, m)`` — src/circulant.jl:1-7, with the
    reference wrapper's defects fixed (it drops W and allocates O like Q)."""
    _require(Q.dim() == 3 and K.dim() == 3 and V.dim() == 3, "circulant_fa expects 3-D arrays")
    _device_check(Q, K, V)
    N, d, B = Q.shape
    O = jl_empty((N, V.shape[1], B), Q.dtype, Q.device)
    l = jl_empty((N, 1, B), torch.float32, Q.device)
    m = jl_empty((N, 1, B), torch.float32, Q.device)
    return circulant_fa_(O, l, m, Q, K, V, W, scale)


def fused_softmax_(P: torch.Tensor, S: torch.Tensor, dims: int = 1) -> torch.Tensor:
    """``fused_softmax!(P, S; dims)`` — src/fused_softmax.jl:1-41 (device versions
    src/cuda/fused_softmax.jl:11-314), in place into P (P may be S).

    S, P: vector (M,), matrix (M, N) or (M, N, batch), Julia column-major;
    dims = 1 normalises columns (first dim), dims = 2 rows (second dim).
    """
    _require(dims in (1, 2), "only softmax in dims 1 or 2 supported")
    _require(S.dim() in (1, 2, 3) and P.shape == S.shape, "P and S must have the same 1-, 2- or 3-D shape")
    _require(S.dim() >= 2 or dims == 1, "a vector is softmaxed along dims = 1")
    shp = tuple(S.shape) + (1,) * (3 - S.dim())
    M, N, B = shp
    code = _dtype_code(S, P)
    _device_check(S, P)
    _require(is_jl_contiguous(S) and is_jl_contiguous(P), "S and P must be Julia column-major contiguous")
    ws = lib().fa_softmax_workspace(M, N, B, dims)
    buf = _workspace(S.device, ws) if ws else None
    _check(lib().fa_softmax(code, _ptr(S), _ptr(P), M, N, B, dims, _ptr(buf), ws, _stream(S)))
    return P


def fused_softmax(S: torch.Tensor, dims: int = 1) -> torch.Tensor:
    """``fused_softmax(S; dims=1)`` — src/fused_softmax.jl:1."""
    P = torch.empty_strided(S.shape, S.stride(), dtype=S.dtype, device=S.device)
    return fused_softmax_(P, S, dims)


def dense_fa_backward(Q, K, V, O, dO, l, m, scale: float = 0.0):
    """``dense_fa_backward(Q, K, V, O, dO, l, m) -> (dQ, dK, dV)`` —
    src/dense.jl:104-167 (executable spec src_cpp/FlashAttention.cpp:194-252).
    The single-pass kernel needs no co-residency of a slab's workgroups, so calls on
    several streams, or processes sharing one GPU, take it as well."""
    for t in (Q, K, V, O, dO, l, m):
        _require(t.dim() == 3, "dense_fa_backward expects 3-D (N, d, batch) arrays")
    N, d, B = Q.shape
    Nk, dv = K.shape[0], V.shape[1]
    _require(K.shape == (Nk, d, B) and V.shape == (Nk, dv, B), "K, V shapes disagree with Q")
    _require(O.shape == (N, dv, B) and dO.shape == (N, dv, B), "O, dO must be (N, dv, batch)")
    _require(l.shape == (N, 1, B) and m.shape == (N, 1, B), "l, m must be (N, 1, batch)")
    _require(l.dtype == torch.float32 and m.dtype == torch.float32, "l, m must be float32")
    code = _dtype_code(Q, K, V, O, dO)
    _device_check(Q, K, V, O, dO, l, m)
    dQ = jl_empty((N, d, B), Q.dtype, Q.device)
    dK = jl_empty((Nk, d, B), Q.dtype, Q.device)
    dV = jl_empty((Nk, dv, B), Q.dtype, Q.device)
    L = lib()
    nws = L.fa_dense_bwd_workspace(code, N, Nk, d, dv, B)
    ws = _workspace(Q.device, nws, entry="dense_fa_backward")
    _check(L.fa_dense_bwd(code, _ptr(Q), _ptr(K), _ptr(V), _ptr(O), _ptr(dO), _ptr(l), _ptr(m),
                          _ptr(dQ), _ptr(dK), _ptr(dV), N, Nk, d, dv, B, float(scale),
                          _ptr(ws), int(nws), _stream(Q)))
    return dQ, dK, dV


def backward_handoff_status(device=None) -> int:
    """fa_dense_bwd_handoff_status for the most recent :func:`dense_fa_backward`
    on the current stream of ``device`` (its workspace is this module's per-stream
    scratch buffer).  Synchronises that stream.  -1: the two-pass form ran (no
    hand-off); 0: single pass, every dQ hand-off completed; 1: some slab's hand-off
    gave up (the whole launch published nothing for 100 ms: a safety net, never
    expected — every wait is on an earlier-dispatched workgroup) and that slab's dQ was
    recomputed by the guarded pass (same values within rounding, other bits, slower).
    Raises FlashAttentionError when no dense_fa_backward
    has run on this stream, or when another entry point has taken the scratch buffer
    since (the module records the last entry point per (device, stream))."""
    device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    stream = torch.cuda.current_stream(device)
    key = (device.type, device.index, stream.cuda_stream)
    buf = _WS.get(key)
    _require(buf is not None and _WS_LAST.get(key) == "dense_fa_backward",
             "the last call that used this stream's scratch buffer was not dense_fa_backward")
    st = ctypes.c_int(-2)
    _check(lib().fa_dense_bwd_handoff_status(_ptr(buf), buf.numel(), ctypes.c_void_p(stream.cuda_stream),
                                             ctypes.byref(st)))
    return int(st.value)


def backward_handoff_trips(device=None) -> int:
    """Slabs whose single-pass dQ hand-off gave up, counted over EVERY dense_fa_backward
    that has used this stream's scratch buffer (a counter in the workspace header that
    no call resets; it starts at whatever the buffer held, so read it before and after
    a series of calls and take the difference).  Synchronises the stream.  Raises
    FlashAttentionError when the last user of the buffer was not dense_fa_backward, when
    the header is not a backward header, or when the buffer was reallocated since the
    first read on this stream (the count would have restarted: a difference across the
    regrowth would be meaningless)."""
    return _backward_header_word(2, device)


_BWD_HDR_MAGIC = 0x46414200   # kBwdHdrMagic (fa_bwd.hip): "FAB\0" | plan in the low byte
_HDR_PTR = {}                  # (device, stream) -> data_ptr of the scratch buffer at the first header read


def _backward_header_word(i: int, device=None) -> int:
    """Word i of the fa_dense_bwd workspace header on this stream's scratch buffer
    (2: the sticky give-up count; 3: the last call left some wrapped slice's A + B to
    the guarded dQ pass — tests; meaningful only after a single-pass call).
    Synchronises the stream.  Checks as backward_handoff_trips says."""
    device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    stream = torch.cuda.current_stream(device)
    key = (device.type, device.index, stream.cuda_stream)
    buf = _WS.get(key)
    _require(buf is not None, "no scratch buffer on this stream yet")
    _require(_WS_LAST.get(key) == "dense_fa_backward",
             "the last call that used this stream's scratch buffer was not dense_fa_backward")
    first = _HDR_PTR.setdefault(key, buf.data_ptr())
    _require(first == buf.data_ptr(),
             "the scratch buffer was reallocated since the first header read on this stream "
             "(its sticky counters restarted)")
    off = ((buf.data_ptr() + 255) & ~255) - buf.data_ptr()
    stream.synchronize()
    words = [int(w) & 0xFFFFFFFF for w in buf[off:off + 16].view(torch.int32).tolist()]
    _require((words[0] & 0xFFFFFF00) == _BWD_HDR_MAGIC, "the scratch buffer holds no fa_dense_bwd header")
    if i == 3:
        _require((words[0] & 0xFF) == 1, "header word 3 is defined only after a single-pass backward")
    return words[i]


# ----------------------------------------------------------------------------
# windowed
# ----------------------------------------------------------------------------
def window_geometry(spatial: Sequence[int], ws: int, stride: int, pad: int):
    """Windows per spatial dim of NNlib.unfold (src/utils.jl:40)."""
    out = tuple((s + 2 * pad - ws) // stride + 1 for s in spatial)
    _require(all(o >= 1 for o in out), "window larger than the padded input")
    return out


_WS = {}
_WS_LAST = {}   # (device, stream) -> name of the entry point that last took the scratch buffer


def _workspace(device, nbytes: int, entry: str = "other") -> torch.Tensor:
    """Scratch buffer for the C ABI's workspace arguments, one per (device,
    stream), grown on demand.

    Keyed by the caller's current stream: two calls on different streams never
    share scratch (split-KV partials, padded K / V copies, windowed / backward
    scratch).  The buffer is allocated while that stream is current, so the
    caching allocator ties it to that stream: when it is replaced by a larger
    one, the old block is only handed out again to work ordered after the
    kernels already queued on that stream (stream-ordered reuse), and calls on
    one stream run in order, so reusing it across calls is safe."""
    stream = torch.cuda.current_stream(device)
    key = (device.type, device.index, stream.cuda_stream)
    _WS_LAST[key] = entry
    buf = _WS.get(key)
    if buf is None or buf.numel() < max(int(nbytes), 1):
        with torch.cuda.stream(stream):
            buf = torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=device)
        _WS[key] = buf
    return buf


def _i64_array(xs):
    arr = (ctypes.c_int64 * len(xs))(*[int(x) for x in xs])
    return arr


def windowed_fa(q, k, v, windowsize: int, stride: Optional[int] = None,
                pad: Optional[int] = None, scale: float = 0.0):
    """``windowed_fa(q, k, v, ws; stride=ws, pad=(ws-1)÷2) -> (y, l, m)`` —
    src/windowed.jl:3-23, fused on the device.

    q, k: (S..., d, B); v: (S..., dv, B); y: (S..., dv, B) with NaN where no
    window covers a pixel (as the reference); l, m: (ws^k, 1, L, B) float32.
    """
    stride = windowsize if stride is None else int(stride)
    pad = (windowsize - 1) // 2 if pad is None else int(pad)
    D = q.dim()
    _require(D >= 3 and k.dim() == D and v.dim() == D, "q, k, v must share rank >= 3")
    nsp = D - 2
    _require(1 <= nsp <= 3, "1 to 3 spatial dims supported")
    sp = tuple(q.shape[:nsp])
    d, B = q.shape[D - 2], q.shape[D - 1]
    dv = v.shape[D - 2]
    _require(tuple(k.shape) == tuple(q.shape), "k must have q's shape")
    _require(tuple(v.shape[:nsp]) == sp and v.shape[D - 1] == B, "v must share q's spatial dims and batch")
    outs = window_geometry(sp, windowsize, stride, pad)
    code = _dtype_code(q, k, v)
    _device_check(q, k, v)
    T = windowsize ** nsp
    L = math.prod(outs)
    y = jl_empty(sp + (dv, B), q.dtype, q.device)
    lw = jl_empty((T, 1, L, B), torch.float32, q.device)
    mw = jl_empty((T, 1, L, B), torch.float32, q.device)
    Lb = lib()
    spa = _i64_array(sp)
    nws = Lb.fa_windowed_fwd_workspace(code, nsp, spa, d, dv, B, windowsize, stride, pad)
    ws = _workspace(q.device, nws)
    _check(Lb.fa_windowed_fwd(code, _ptr(q), _ptr(k), _ptr(v), _ptr(y), _ptr(lw), _ptr(mw),
                              nsp, spa, d, dv, B, windowsize, stride, pad,
                              float(scale), _ptr(ws), int(nws), _stream(q)))
    return y, lw, mw


def _window_args(spatial, windowsize, stride, pad):
    stride = windowsize if stride is None else int(stride)
    pad = (windowsize - 1) // 2 if pad is None else int(pad)
    nsp = len(spatial)
    _require(1 <= nsp <= 3, "1 to 3 spatial dims supported")
    outs = window_geometry(spatial, windowsize, stride, pad)
    return stride, pad, nsp, outs


def window(x: torch.Tensor, windowsize: int, stride: Optional[int] = None,
           pad: Optional[int] = None) -> torch.Tensor:
    """``window(x, ws; stride=ws, pad=(ws-1)÷2)`` — src/utils.jl:36-45
    (NNlib.unfold) on the device: x (S..., C, B) -> (ws^k, C, L, B), zero padding."""
    D = x.dim()
    _require(D >= 3, "x must have rank >= 3: (spatial..., C, B)")
    sp = tuple(x.shape[:D - 2])
    C, B = x.shape[D - 2], x.shape[D - 1]
    stride, pad, nsp, outs = _window_args(sp, windowsize, stride, pad)
    code = _dtype_code(x)
    _device_check(x)
    X = jl_empty((windowsize ** nsp, C, math.prod(outs), B), x.dtype, x.device)
    _check(lib().fa_window(code, _ptr(x), _ptr(X), nsp, _i64_array(sp), C, B, windowsize, stride, pad,
                           _stream(x)))
    return X


def unwindow(X: torch.Tensor, outputsize: Sequence[int], windowsize: int, stride: Optional[int] = None,
             pad: Optional[int] = None) -> torch.Tensor:
    """``unwindow(X, outputsize, ws; stride, pad)`` — src/utils.jl:47-54
    (NNlib.fold): (ws^k, C, L, B) -> outputsize = (S..., C, B), overlapping
    window contributions SUMMED (0 where no window covers a pixel)."""
    outputsize = tuple(int(o) for o in outputsize)
    _require(len(outputsize) >= 3 and X.dim() == 4, "X: (ws^k, C, L, B); outputsize: (spatial..., C, B)")
    sp = outputsize[:-2]
    C, B = outputsize[-2], outputsize[-1]
    stride, pad, nsp, outs = _window_args(sp, windowsize, stride, pad)
    _require(tuple(X.shape) == (windowsize ** nsp, C, math.prod(outs), B),
             f"X has shape {tuple(X.shape)}, the geometry needs {(windowsize ** nsp, C, math.prod(outs), B)}")
    code = _dtype_code(X)
    _device_check(X)
    x = jl_empty(outputsize, X.dtype, X.device)
    _check(lib().fa_unwindow(code, _ptr(X), _ptr(x), nsp, _i64_array(sp), C, B, windowsize, stride, pad,
                             _stream(X)))
    return x


def _rm(t: torch.Tensor) -> torch.Tensor:
    """Row-major view (reversed dims) of a Julia column-major tensor: same memory."""
    return t.permute(*range(t.dim() - 1, -1, -1))


def jl_reshape(t: torch.Tensor, shape: Sequence[int]) -> torch.Tensor:
    """Julia ``reshape`` (column-major order) of a column-major contiguous tensor: a view."""
    _require(is_jl_contiguous(t), "jl_reshape needs a Julia column-major contiguous tensor")
    return _rm(_rm(t).reshape(tuple(int(x) for x in reversed(tuple(shape)))))


def dense_dpa(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, scale: float = 0.0):
    """``dense_dpa(q, k, v) -> (y, P)`` — src/naive/dense.jl:1-35, the reference's
    materialising attention (its test oracle for dense_fa, test/test.jl:19):
    P = softmax(τ Q Kᵀ; dims=2) as an (N, Nk, B) array, y = P V.

    The two products are plain library GEMMs (hipBLASLt through torch.bmm on
    the column-major views; no transpose copies), the softmax is this
    library's fa_softmax kernel (dims = 2).  P is in the input dtype, as the
    reference computes it in T.  Memory is O(N·Nk·B): use dense_fa for size."""
    D = q.dim()
    _require(D >= 3 and k.dim() == D and v.dim() == D, "q, k, v must share rank >= 3")
    dqk, B = q.shape[D - 2], q.shape[D - 1]
    dvo = v.shape[D - 2]
    _require(k.shape[D - 2] == dqk and k.shape[D - 1] == B and v.shape[D - 1] == B,
             "DimensionMismatch: k must match q's feature and batch dims, v the batch dim")
    _dtype_code(q, k, v)
    _device_check(q, k, v)
    _require(all(is_jl_contiguous(t) for t in (q, k, v)), "q, k, v must be Julia column-major contiguous")
    N = math.prod(q.shape[:D - 2])
    Nk = math.prod(k.shape[:D - 2])
    _require(math.prod(v.shape[:D - 2]) == Nk, "DimensionMismatch: v must have k's token count")
    tau = float(scale) if scale > 0 else 1.0 / math.sqrt(dqk)
    Qr = _rm(q).reshape(B, dqk, N)           # column-major (N, d, B) = row-major [B][d][N]
    Kr = _rm(k).reshape(B, dqk, Nk)
    Vr = _rm(v).reshape(B, dvo, Nk)
    St = torch.bmm(Kr.transpose(1, 2), Qr)  # [B][Nk][N] = column-major (N, Nk, B): P's layout
    St.mul_(tau)
    P = _rm(St)                               # (N, Nk, B) view
    fused_softmax_(P, P, dims=2)
    Y = torch.bmm(Vr, St)                     # [B][dv][N] = column-major (N, dv, B)
    y = jl_reshape(_rm(Y), tuple(q.shape[:D - 2]) + (dvo, B))
    return y, P


def windowed_dpa(q, k, v, windowsize: int, stride: Optional[int] = None, pad: Optional[int] = None):
    """``windowed_dpa(q, k, v, ws; stride, pad) -> (y, P)`` — src/naive/windowed.jl:3-22:
    window (fa_window) → dense_dpa over the (ws^k, d, L·B) window batch →
    unwindow (fa_unwindow) ÷ coverage (unwindow of windowed ones, :16-17).
    P: (ws^k, ws^k, L, B).  Uncovered pixels are 0/0 = NaN, as the reference."""
    D = q.dim()
    sp = tuple(q.shape[:D - 2])
    dvo, B = v.shape[D - 2], v.shape[D - 1]
    stride, pad, nsp, outs = _window_args(sp, windowsize, stride, pad)
    qw, kw, vw = (window(a, windowsize, stride, pad) for a in (q, k, v))
    T, L = windowsize ** nsp, math.prod(outs)
    yw, Pw = dense_dpa(*(jl_reshape(a, (T, a.shape[1], L * B)) for a in (qw, kw, vw)))
    szy = sp + (dvo, B)
    ones = jl_empty(szy, v.dtype, v.device).fill_(1)
    divisor = unwindow(window(ones, windowsize, stride, pad), szy, windowsize, stride, pad)
    y = unwindow(jl_reshape(yw, (T, dvo, L, B)), szy, windowsize, stride, pad)
    y.div_(divisor)
    return y, jl_reshape(Pw, (T, T, L, B))


def circulant_band_index(N: int, W: int, device="cuda") -> torch.Tensor:
    """0-based key index J[w, i] of band entry w of query i, in the reference's
    order: ``cartesian_circulant((i-1)*W + w, N, W)[1]`` (src/utils.jl:6-17, used
    by src/naive/circulant.jl:21-22 and src/circulant.jl:74-75), vectorised.
    The keys of query i are (i − p + t) mod N, t < W, p = (W−1)÷2; the reference's
    circshift only rotates their order for the first and last p columns."""
    p = (W - 1) // 2
    i = torch.arange(N, device=device, dtype=torch.int64)[None, :]
    w = torch.arange(W, device=device, dtype=torch.int64)[:, None]
    j1 = i + 1                                            # 1-based column
    m0 = torch.where(j1 <= p, torch.remainder(w - i + p, W),
                     torch.where(j1 > N - p, torch.remainder(w - p + N - i - 1, W), w.expand(W, N)))
    return torch.remainder(m0 + i - p, N)


def circulant_dpa(Q: torch.Tensor, K: torch.Tensor, V: torch.Tensor, W: int, scale: float = 0.0):
    """``circulant_dpa(Q, K, V, W) -> (O, P)`` — src/naive/circulant.jl:1-36, the
    reference's materialising banded attention (its check for circulant_fa,
    bench/compare.jl:72-74): band scores P[w, i, b] = τ qᵢ·k_J[w,i] (:19-24),
    softmax over the band (dims = 1, this library's fa_softmax kernel, :27),
    O = Σ_w P[w, i] v_J[w,i] (:28-34).

    Representation deviation: the reference returns P as the transposed sparse
    circulant matrix (``batch_circulant(P) |> transpose``, :28); this returns its
    nonzeros, the (W, N, B) band array the reference builds it from, in the same
    entry order.  Gathers and reductions are torch ops on the device; memory is
    O(W·N·d·B)."""
    _require(Q.dim() == 3 and K.dim() == 3 and V.dim() == 3, "circulant_dpa expects 3-D (N, d, batch) arrays")
    N, d, B = Q.shape
    dv = V.shape[1]
    _require(K.shape == (N, d, B) and V.shape == (N, dv, B), "DimensionMismatch: K must match Q, V (N, dv, batch)")
    _require(int(W) >= 1, "DimensionMismatch: window size W must be >= 1")
    _dtype_code(Q, K, V)
    _device_check(Q, K, V)
    W = int(W)
    tau = float(scale) if scale > 0 else 1.0 / math.sqrt(d)
    J = circulant_band_index(N, W, Q.device)              # (W, N)
    Qr, Kr, Vr = _rm(Q), _rm(K), _rm(V)                   # [B][d][N], [B][d][N], [B][dv][N]
    acc = torch.float64 if Q.dtype == torch.float64 else torch.float32
    S = (Kr[:, :, J].to(acc) * Qr[:, :, None, :].to(acc)).sum(1) * tau    # [B][W][N]
    P = jl_empty((W, N, B), Q.dtype, Q.device)
    _rm(P).copy_(S.transpose(1, 2))                       # column-major (W, N, B) = [B][N][W]
    fused_softmax_(P, P, dims=1)
    Pw = _rm(P).transpose(1, 2).to(acc)                   # [B][W][N]
    O = jl_empty((N, dv, B), Q.dtype, Q.device)
    _rm(O).copy_((Vr[:, :, J].to(acc) * Pw[:, None, :, :]).sum(2))   # [B][dv][N]
    return O, P


def block_dpa(q, k, v, windowsize: int):
    """``block_dpa(q, k, v, ws) = windowed_dpa(q, k, v, ws)`` — src/naive/windowed.jl:1
    (the reference passes no keywords: stride = ws, pad = (ws-1)÷2)."""
    return windowed_dpa(q, k, v, windowsize)


def block_fa(q, k, v, windowsize: int, pad: int = 0, scale: float = 0.0):
    """``block_fa(q, k, v, ws; pad=0)`` = windowed_fa with stride = ws — src/windowed.jl:1."""
    return windowed_fa(q, k, v, windowsize, stride=windowsize, pad=pad, scale=scale)


def windowed_fa_backward(q, k, v, y, dy, l, m, windowsize: int, stride: Optional[int] = None,
                         pad: Optional[int] = None, scale: float = 0.0):
    """Backward of :func:`windowed_fa`: returns (dq, dk, dv)."""
    stride = windowsize if stride is None else int(stride)
    pad = (windowsize - 1) // 2 if pad is None else int(pad)
    D = q.dim()
    _require(D >= 3 and all(t.dim() == D for t in (k, v, y, dy)), "q, k, v, y, dy must share rank >= 3")
    nsp = D - 2
    _require(1 <= nsp <= 3, "1 to 3 spatial dims supported")
    sp = tuple(q.shape[:nsp])
    d, B = q.shape[D - 2], q.shape[D - 1]
    dv = v.shape[D - 2]
    _require(tuple(k.shape) == tuple(q.shape), "k must have q's shape")
    _require(tuple(v.shape[:nsp]) == sp and v.shape[D - 1] == B, "v must share q's spatial dims and batch")
    _require(tuple(y.shape) == sp + (dv, B) and tuple(dy.shape) == sp + (dv, B),
             f"y and dy must be {sp + (dv, B)}")
    outs = window_geometry(sp, windowsize, stride, pad)
    T, L = windowsize ** nsp, math.prod(outs)
    _require(tuple(l.shape) == (T, 1, L, B) and tuple(m.shape) == (T, 1, L, B),
             f"l, m must be {(T, 1, L, B)} (the forward's window statistics)")
    _require(l.dtype == torch.float32 and m.dtype == torch.float32, "l, m must be float32")
    code = _dtype_code(q, k, v, y, dy)
    _device_check(q, k, v, y, dy, l, m)
    dq = jl_empty(sp + (d, B), q.dtype, q.device)
    dk = jl_empty(sp + (d, B), q.dtype, q.device)
    dvv = jl_empty(sp + (dv, B), q.dtype, q.device)
    Lb = lib()
    spa = _i64_array(sp)
    nws = Lb.fa_windowed_workspace(code, nsp, spa, d, dv, B, windowsize, stride, pad)
    ws = _workspace(q.device, nws)
    _check(Lb.fa_windowed_bwd(code, _ptr(q), _ptr(k), _ptr(v), _ptr(y), _ptr(dy), _ptr(l), _ptr(m),
                              _ptr(dq), _ptr(dk), _ptr(dvv), nsp, spa, d, dv, B, windowsize,
                              stride, pad, float(scale), _ptr(ws), int(nws), _stream(q)))
    return dq, dk, dvv
