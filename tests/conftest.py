"""Shared test configuration.

Markers: ``gpu`` — needs a ROCm device (MI355X); run with ``-m gpu``.
Everything else runs on CPU (``-m "not gpu"``).

Tolerance policy (applied to device outputs vs the float64
oracle on identical, bf16-representable inputs):
  fp32 output : norm-wise ‖x−y‖ ≤ √eps(Float32)·max(‖x‖,‖y‖)  (Julia ≈, the
                reference's own check, test/test.jl:19-20) AND elementwise
                |x−y| ≤ 1e-5·max|y| + 1e-6.
  bf16 output : elementwise |x−y| ≤ 2e-2·(1+|y|) and norm-wise rel ≤ 1e-2.
  fp16 output : elementwise |x−y| ≤ 5e-3·(1+|y|) and norm-wise rel ≤ 3e-3.
  l, m (fp32) : |Δ| ≤ rtol·(1+|y|) with rtol 1e-5 (fp32 inputs) / 1e-4 (16-bit).
"""
from __future__ import annotations

import glob
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "flashattention.jl_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X)")


def golden_files(prefix: str):
    return sorted(glob.glob(os.path.join(GOLDEN, prefix + "*.npz")))


def bits_to_f64(bits: np.ndarray) -> np.ndarray:
    return (bits.astype(np.uint32) << 16).view(np.float32).astype(np.float64)


def load_golden(path: str) -> dict:
    z = np.load(path, allow_pickle=False)
    out = {}
    for k in z.files:
        out[k[3:] if k.startswith("in_") else k] = (
            bits_to_f64(z[k]) if k.startswith("in_") else z[k])
    return out


TOL = {
    "float32": dict(norm=np.sqrt(np.finfo(np.float32).eps), elem_rel_max=1e-5, elem_abs=1e-6, lm=1e-5),
    "bfloat16": dict(norm=1e-2, elem=2e-2, lm=1e-4),
    "float16": dict(norm=3e-3, elem=5e-3, lm=1e-4),
}


def assert_close(x, y, dtype: str, what: str = "", nan_ok: bool = False):
    """Device output x vs oracle y (float64) under the policy above."""
    x = np.asarray(x, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    assert x.shape == y.shape, f"{what}: shape {x.shape} vs {y.shape}"
    if nan_ok:
        nx, ny = np.isnan(x), np.isnan(y)
        assert np.array_equal(nx, ny), f"{what}: NaN pattern differs ({nx.sum()} vs {ny.sum()})"
        x = np.where(nx, 0.0, x)
        y = np.where(ny, 0.0, y)
    assert np.all(np.isfinite(x)), f"{what}: non-finite values"
    t = TOL[dtype]
    dn = np.linalg.norm(x - y)
    ref = max(np.linalg.norm(x), np.linalg.norm(y), 1e-30)
    assert dn <= t["norm"] * ref, f"{what}: norm-wise rel err {dn / ref:.3e} > {t['norm']:.1e}"
    err = np.abs(x - y)
    if dtype == "float32":
        lim = t["elem_rel_max"] * np.max(np.abs(y)) + t["elem_abs"]
        assert err.max() <= lim, f"{what}: max abs err {err.max():.3e} > {lim:.3e}"
    else:
        bad = err > t["elem"] * (1 + np.abs(y))
        assert not bad.any(), f"{what}: {bad.sum()} elements beyond {t['elem']}·(1+|y|), worst {err.max():.3e}"


def assert_lm_close(x, y, dtype: str, what: str = ""):
    x = np.asarray(x, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    assert x.shape == y.shape, f"{what}: shape {x.shape} vs {y.shape}"
    rtol = TOL[dtype]["lm"]
    err = np.abs(x - y) / (1 + np.abs(y))
    assert err.max() <= rtol, f"{what}: rel err {err.max():.3e} > {rtol:.1e}"
