"""CPU tests of the C-ABI boundary: libfa_hip.so loads, exports every symbol
include/fa_hip.h declares, and rejects bad arguments with the documented
status codes and thread-local messages BEFORE touching the device (so these
run without a GPU).  Plus the Python mirror's argument checking."""
from __future__ import annotations

import ctypes
import os
import re
import threading

import pytest
import torch

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "fa_hip.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\**\s+\**(fa_\w+)\s*\(", src, flags=re.M)))


def test_header_declares_the_boundary():
    fns = declared_functions()
    for f in ("fa_dense_fwd", "fa_dense_bwd", "fa_dense_bwd_workspace", "fa_windowed_fwd",
              "fa_windowed_fwd_workspace", "fa_windowed_bwd", "fa_windowed_workspace",
              "fa_circulant_fwd", "fa_softmax", "fa_softmax_workspace",
              "fa_last_error", "fa_abi_version", "fa_max_head_dim"):
        assert f in fns


def test_header_states_the_kernels_give_up_bound():
    """The boundary contract's hand-off give-up bound is the one bwd_fused implements:
    fa_bwd.hip takes kStallUs from the header's macro, and the prose around it states
    the same figure (in ms) and the no-progress rule (INTEGRATION.md agrees)."""
    hdr = open(HEADER).read()
    m = re.search(r"#define\s+FA_BWD_HANDOFF_STALL_US\s+(\d+)", hdr)
    assert m, "FA_BWD_HANDOFF_STALL_US missing from fa_hip.h"
    us = int(m.group(1))
    src = open(os.path.join(ROOT, "flashattention.jl_amd", "csrc", "fa_bwd.hip")).read()
    k = re.search(r"constexpr\s+int\s+kStallUs\s*=\s*(\w+)\s*;", src)
    assert k and k.group(1) in ("FA_BWD_HANDOFF_STALL_US", str(us)), "kStallUs does not follow the header"
    prose = re.sub(r"\s+", " ", hdr)
    assert f"({us // 1000} ms)" in prose and "made progress" in prose
    assert "50 us" not in prose and "20 ms" not in prose
    integ = re.sub(r"\s+", " ", open(os.path.join(ROOT, "INTEGRATION.md")).read())
    assert f"{us // 1000} ms" in integ


def test_library_loads_and_exports_every_declared_symbol():
    import fa_hip
    L = fa_hip.lib()
    for f in declared_functions():
        assert hasattr(L, f), f"{f} declared in fa_hip.h but not exported"
    assert L.fa_abi_version() == 1
    assert L.fa_max_head_dim() == 128


def test_exports_are_c_symbols_not_mangled():
    import subprocess
    import fa_hip
    out = subprocess.run(["nm", "-D", "--defined-only", fa_hip.lib_path()], capture_output=True,
                         text=True, check=True).stdout
    syms = {line.split()[-1] for line in out.splitlines() if line.strip()}
    for f in declared_functions():
        assert f in syms


def test_product_library_carries_no_diagnostic_hooks():
    # the phase-stamp reader and the timing-only ablation modes exist only in
    # -DFA_BWD_STAMP4 / -DFA_BWD_ABL builds (tools/exp), never in the shipped library
    import subprocess
    import fa_hip
    out = subprocess.run(["nm", "-D", "--defined-only", fa_hip.lib_path()], capture_output=True,
                         text=True, check=True).stdout
    syms = {line.split()[-1] for line in out.splitlines() if line.strip()}
    assert "fa_debug_bwd_stamps" not in syms
    L = fa_hip.lib()
    old = L.fa_debug_set_bwd_mode(0)
    try:
        assert L.fa_debug_set_bwd_mode(5) == -1, "timing-only ablation modes accepted by the product build"
    finally:
        L.fa_debug_set_bwd_mode(old)


def _i(x):
    return ctypes.c_int64(x)


def test_invalid_arguments_return_status_and_message():
    import fa_hip
    L = fa_hip.lib()
    P = ctypes.c_void_p(16)  # never dereferenced: validation fails first
    # unknown dtype
    rc = L.fa_dense_fwd(9, P, P, P, P, P, P, 4, 4, 4, 4, 1, 0.0, None)
    assert rc == fa_hip.FA_ERR_INVALID_ARG and b"dtype" in L.fa_last_error()
    # negative sizes / empty head dims → DimensionMismatch
    rc = L.fa_dense_fwd(1, P, P, P, P, P, P, -1, 4, 4, 4, 1, 0.0, None)
    assert rc == fa_hip.FA_ERR_INVALID_ARG and b"DimensionMismatch" in L.fa_last_error()
    rc = L.fa_dense_fwd(1, P, P, P, P, P, P, 4, 4, 0, 4, 1, 0.0, None)
    assert rc == fa_hip.FA_ERR_INVALID_ARG and b"DimensionMismatch" in L.fa_last_error()
    # empty inputs (N = 0 or batch = 0) are a no-op, as dense_fa! runs no tile
    # (src/dense.jl:45): nothing is dereferenced or launched
    assert L.fa_dense_fwd(1, None, None, None, None, None, None, 0, 4, 4, 4, 1, 0.0, None) == 0
    assert L.fa_dense_fwd(1, None, None, None, None, None, None, 4, 4, 4, 4, 0, 0.0, None) == 0
    # empty batch in the windowed / circulant / softmax entries: validated, then a
    # no-op (the reference loops over zero images / rows / slabs)
    sp2 = (ctypes.c_int64 * 2)(16, 16)
    assert L.fa_windowed_fwd(1, None, None, None, None, None, None, 2, sp2, 8, 8, 0, 7, 7, 3,
                             0.0, None, 0, None) == 0
    assert L.fa_windowed_bwd(1, None, None, None, None, None, None, None, None, None, None, 2, sp2,
                             8, 8, 0, 7, 7, 3, 0.0, None, 0, None) == 0
    assert L.fa_window(1, None, None, 2, sp2, 8, 0, 7, 7, 3, None) == 0
    assert L.fa_unwindow(1, None, None, 2, sp2, 8, 0, 7, 7, 3, None) == 0
    rc = L.fa_windowed_fwd(1, None, None, None, None, None, None, 2, sp2, 8, 8, 0, 17, 17, 0,
                           0.0, None, 0, None)
    assert rc == fa_hip.FA_ERR_INVALID_ARG and b"window" in L.fa_last_error()
    assert L.fa_circulant_fwd(1, None, None, None, None, None, None, 0, 32, 32, 1, 5, 0.0, None) == 0
    assert L.fa_circulant_fwd(1, None, None, None, None, None, None, 64, 32, 32, 0, 5, 0.0, None) == 0
    assert L.fa_softmax(1, None, None, 8, 8, 0, 1, None, 0, None) == 0
    rc = L.fa_softmax(1, None, None, 0, 8, 1, 1, None, 0, None)
    assert rc == fa_hip.FA_ERR_INVALID_ARG and b"DimensionMismatch" in L.fa_last_error()
    # null pointer
    rc = L.fa_dense_fwd(1, None, P, P, P, P, P, 4, 4, 4, 4, 1, 0.0, None)
    assert rc == fa_hip.FA_ERR_INVALID_ARG and b"null" in L.fa_last_error()
    # unsupported head dim
    rc = L.fa_dense_fwd(1, P, P, P, P, P, P, 4, 4, 129, 4, 1, 0.0, None)
    assert rc == fa_hip.FA_ERR_UNSUPPORTED and b"head dimension" in L.fa_last_error()
    # windowed: window larger than padded input
    sp = (ctypes.c_int64 * 2)(5, 5)
    rc = L.fa_windowed_fwd(1, P, P, P, P, P, P, 2, sp, 4, 4, 1, 9, 9, 0, 0.0, None, 0, None)
    assert rc == fa_hip.FA_ERR_INVALID_ARG and b"window" in L.fa_last_error()
    rc = L.fa_windowed_fwd(1, P, P, P, P, P, P, 4, sp, 4, 4, 1, 3, 3, 0, 0.0, None, 0, None)
    assert rc == fa_hip.FA_ERR_INVALID_ARG and b"nspatial" in L.fa_last_error()
    # circulant: band width and head dim validated before any launch
    rc = L.fa_circulant_fwd(1, P, P, P, P, P, P, 64, 32, 32, 1, 0, 0.0, None)
    assert rc == fa_hip.FA_ERR_INVALID_ARG and b"window size" in L.fa_last_error()
    rc = L.fa_circulant_fwd(1, P, P, P, P, P, P, 64, 129, 32, 1, 7, 0.0, None)
    assert rc == fa_hip.FA_ERR_UNSUPPORTED and b"head dimension" in L.fa_last_error()
    rc = L.fa_circulant_fwd(1, P, None, P, P, P, P, 64, 32, 32, 1, 7, 0.0, None)
    assert rc == fa_hip.FA_ERR_INVALID_ARG and b"null" in L.fa_last_error()
    # softmax: dims, sizes and the long-column workspace are checked before any launch
    rc = L.fa_softmax(1, P, P, 8, 8, 1, 3, None, 0, None)
    assert rc == fa_hip.FA_ERR_INVALID_ARG and b"dims" in L.fa_last_error()
    rc = L.fa_softmax(1, P, P, 0, 8, 1, 1, None, 0, None)
    assert rc == fa_hip.FA_ERR_INVALID_ARG and b"DimensionMismatch" in L.fa_last_error()
    assert L.fa_softmax_workspace(8192, 4, 1, 1) == 0 and L.fa_softmax_workspace(8193, 4, 1, 1) > 0
    assert L.fa_softmax_workspace(100000, 4, 1, 2) == 0
    rc = L.fa_softmax(1, P, P, 100000, 4, 1, 1, None, 0, None)
    assert rc == fa_hip.FA_ERR_WORKSPACE
    # backward: workspace check happens before any launch
    need = L.fa_dense_bwd_workspace(1, 128, 128, 64, 64, 2)
    if need > 0:
        rc = L.fa_dense_bwd(1, P, P, P, P, P, P, P, P, P, P, 128, 128, 64, 64, 2, 0.0, None, 0, None)
        assert rc == fa_hip.FA_ERR_WORKSPACE


def test_last_error_is_thread_local():
    import fa_hip
    L = fa_hip.lib()
    P = ctypes.c_void_p(16)
    assert L.fa_dense_fwd(9, P, P, P, P, P, P, 4, 4, 4, 4, 1, 0.0, None) != 0
    seen = {}

    def other():
        seen["msg"] = L.fa_last_error()

    t = threading.Thread(target=other)
    t.start()
    t.join()
    assert seen["msg"] == b""
    assert b"dtype" in L.fa_last_error()


def test_python_mirror_shape_checks_raise_dimension_mismatch():
    import fa_hip
    Q = fa_hip.jl_empty((8, 4, 2), device="cpu")
    K = fa_hip.jl_empty((8, 5, 2), device="cpu")
    O = fa_hip.jl_empty((8, 4, 2), device="cpu")
    l = fa_hip.jl_empty((8, 1, 2), device="cpu")
    with pytest.raises(fa_hip.DimensionMismatch):
        fa_hip.dense_fa_(O, l, l, Q, K, Q)
    with pytest.raises(fa_hip.DimensionMismatch):
        fa_hip.dense_fa_(fa_hip.jl_empty((8, 3, 2), device="cpu"), l, l, Q, Q, Q)
    # correct shapes but host arrays: loud refusal, no CPU fallback
    with pytest.raises(TypeError, match="no CPU fallback"):
        fa_hip.dense_fa_(O, l, l, Q, Q, Q)
    with pytest.raises(fa_hip.DimensionMismatch):
        fa_hip.windowed_fa(fa_hip.jl_empty((4, 4, 2, 1), device="cpu"),
                           fa_hip.jl_empty((4, 4, 2, 1), device="cpu"),
                           fa_hip.jl_empty((4, 4, 2, 1), device="cpu"), 9, stride=9, pad=0)
    with pytest.raises(fa_hip.DimensionMismatch):
        fa_hip.circulant_fa_(O, l, l, Q, K, Q, 3)
    with pytest.raises(fa_hip.DimensionMismatch):
        fa_hip.circulant_fa_(O, l, l, Q, Q, Q, 0)
    with pytest.raises(TypeError, match="no CPU fallback"):
        fa_hip.circulant_fa(Q, Q, Q, 3)


def test_julia_layout_helpers():
    import fa_hip
    t = fa_hip.jl_empty((5, 3, 2), device="cpu")
    assert t.shape == (5, 3, 2) and t.stride() == (1, 5, 15)
    assert fa_hip.is_jl_contiguous(t)
    assert not fa_hip.is_jl_contiguous(torch.empty(5, 3, 2))
    x = torch.arange(30.0).reshape(5, 3, 2)
    assert torch.equal(fa_hip.jl_tensor(x, device="cpu"), x)


def test_workspace_queries_are_positive_and_monotone():
    import fa_hip
    L = fa_hip.lib()
    sp = (ctypes.c_int64 * 2)(128, 128)
    a = L.fa_windowed_workspace(1, 2, sp, 64, 64, 1, 7, 7, 3)
    b = L.fa_windowed_workspace(1, 2, sp, 64, 64, 4, 7, 7, 3)
    assert 0 < a < b
    assert L.fa_windowed_fwd_workspace(1, 2, sp, 64, 64, 1, 7, 7, 3) <= a
    assert L.fa_dense_bwd_workspace(1, 4096, 4096, 64, 64, 64) >= 2 * 4 * 4096 * 64
    assert L.fa_dense_bwd_workspace(9, 4096, 4096, 64, 64, 64) == 0   # bad dtype
