"""ctypes binding of oracle/libfa_cpu.so (the C OpenMP port of dense_fa!,
src/dense.jl:21-102).  TEST INFRASTRUCTURE ONLY (see oracle/__init__.py)."""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "libfa_cpu.so")
        if not os.path.exists(path):
            raise ImportError(f"{path} missing: run `make -C oracle` or __graft_entry__.build()")
        L = ctypes.CDLL(path)
        vp, i64 = ctypes.c_void_p, ctypes.c_int64
        for name in ("fa_cpu_dense_fwd_f32", "fa_cpu_dense_fwd_f64"):
            fn = getattr(L, name)
            fn.restype = ctypes.c_int
            fn.argtypes = [vp, vp, vp, vp, vp, vp, i64, i64, i64, i64, i64, ctypes.c_int]
        for name in ("fa_cpu_dense_fwd_blas_f32", "fa_cpu_dense_fwd_blas_f64"):
            fn = getattr(L, name)
            fn.restype = ctypes.c_int
            fn.argtypes = [vp, vp, vp, vp, vp, vp, i64, i64, i64, i64, i64, ctypes.c_int]
        L.fa_cpu_set_blas.restype = ctypes.c_int
        L.fa_cpu_set_blas.argtypes = [vp, vp, vp]
        L.fa_cpu_max_threads.restype = ctypes.c_int
        _LIB = L
    return _LIB


_BLAS = None


def blas_info() -> str:
    """Load numpy's bundled OpenBLAS (ILP64 CBLAS, scipy_ prefix) and hand its
    sgemm / dgemm / set_num_threads to the C port.  Returns the library path."""
    global _BLAS
    if _BLAS is None:
        import glob
        libdir = os.path.join(os.path.dirname(os.path.dirname(np.__file__)), "numpy.libs")
        cands = sorted(glob.glob(os.path.join(libdir, "libscipy_openblas64_*.so")))
        if not cands:
            raise ImportError(f"no OpenBLAS under {libdir}")
        B = ctypes.CDLL(cands[0])
        addr = lambda n: ctypes.cast(getattr(B, n), ctypes.c_void_p).value
        rc = lib().fa_cpu_set_blas(addr("scipy_cblas_sgemm64_"), addr("scipy_cblas_dgemm64_"),
                                   addr("scipy_openblas_set_num_threads64_"))
        if rc != 0:
            raise ImportError("fa_cpu_set_blas failed")
        _BLAS = (B, cands[0])
    return _BLAS[1]


def dense_fa_blas(Q: np.ndarray, K: np.ndarray, V: np.ndarray, nthreads: int = 0):
    """dense_fa! with the reference's BLAS structure (one gemm per tile product,
    src/dense.jl:77/:88) — see fa_cpu.c.  Same arguments and results as dense_fa."""
    blas_info()
    dt = np.float64 if Q.dtype == np.float64 else np.float32
    Q = np.asfortranarray(Q, dtype=dt)
    K = np.asfortranarray(K, dtype=dt)
    V = np.asfortranarray(V, dtype=dt)
    N, d, B = Q.shape
    Nk, dv = K.shape[0], V.shape[1]
    O = np.empty((N, dv, B), dtype=dt, order="F")
    l = np.empty((N, 1, B), dtype=dt, order="F")
    m = np.empty((N, 1, B), dtype=dt, order="F")
    fn = lib().fa_cpu_dense_fwd_blas_f64 if dt == np.float64 else lib().fa_cpu_dense_fwd_blas_f32
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    rc = fn(p(Q), p(K), p(V), p(O), p(l), p(m), N, Nk, d, dv, B, int(nthreads))
    if rc != 0:
        raise RuntimeError(f"fa_cpu_dense_fwd_blas failed ({rc})")
    return O, l, m


def dense_fa(Q: np.ndarray, K: np.ndarray, V: np.ndarray, nthreads: int = 0):
    """dense_fa!(O, l, m, Q, K, V) on Julia-shaped (N, d, B) arrays.

    Arrays are converted to column-major (Fortran) float32/float64 as needed.
    Returns O (N, dv, B), l, m (N, 1, B) in the input precision."""
    dt = np.float64 if Q.dtype == np.float64 else np.float32
    Q = np.asfortranarray(Q, dtype=dt)
    K = np.asfortranarray(K, dtype=dt)
    V = np.asfortranarray(V, dtype=dt)
    N, d, B = Q.shape
    Nk, dv = K.shape[0], V.shape[1]
    O = np.empty((N, dv, B), dtype=dt, order="F")
    l = np.empty((N, 1, B), dtype=dt, order="F")
    m = np.empty((N, 1, B), dtype=dt, order="F")
    fn = lib().fa_cpu_dense_fwd_f64 if dt == np.float64 else lib().fa_cpu_dense_fwd_f32
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    rc = fn(p(Q), p(K), p(V), p(O), p(l), p(m), N, Nk, d, dv, B, int(nthreads))
    if rc != 0:
        raise RuntimeError(f"fa_cpu_dense_fwd failed ({rc})")
    return O, l, m
