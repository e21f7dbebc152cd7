"""GPU parity tests: standalone fused softmax through the C ABI (fa_softmax) vs
the float64 oracle restatement of fused_softmax! (src/fused_softmax.jl:1-41):
golden vectors × 3 dtypes, both dims on every kernel (register column,
chunked long column, register row, two-pass row), vectors, in-place use and
the reference's special-value semantics.  Tolerances: tests/conftest.py."""
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


@pytest.mark.parametrize("dtype", list(DT))
@pytest.mark.parametrize("path", golden_files("softmax_"), ids=lambda p: p.split("/")[-1][:-4])
def test_softmax_golden(fa, path, dtype):
    g = load_golden(path)
    S = fa.jl_tensor(g["s"], DT[dtype])
    P = fa.fused_softmax(S, int(g["dims"]))
    torch.cuda.synchronize()
    assert fa.is_jl_contiguous(P) and tuple(P.shape) == g["p"].shape
    assert_close(_np(P), g["p"], dtype, "P")


SHAPES = [
    ((4096, 64, 3), 1),      # register column kernel
    ((8192, 2, 1), 1),       # exactly one chunk
    ((50000, 3, 2), 1),      # chunked column kernel (7 chunks)
    ((1000, 32, 2), 2),      # register row kernel (N = 32)
    ((777, 129, 3), 2),      # two-pass row kernel
    ((100000,), 1),          # long vector
]


@pytest.mark.parametrize("dtype", list(DT))
@pytest.mark.parametrize("shape,dims", SHAPES)
def test_softmax_random(fa, shape, dims, dtype):
    rng = np.random.default_rng(sum(shape) + dims)
    Sh = torch.tensor(rng.standard_normal(shape) * 4).to(DT[dtype]).double().numpy()
    P = fa.fused_softmax(fa.jl_tensor(Sh, DT[dtype]), dims)
    torch.cuda.synchronize()
    assert_close(_np(P), O.fused_softmax(Sh, dims), dtype, "P")


@pytest.mark.parametrize("dims", [1, 2])
def test_softmax_in_place(fa, dims):
    """fused_softmax!(S) = fused_softmax!(S, S) (src/fused_softmax.jl:2)."""
    rng = np.random.default_rng(9)
    Sh = rng.standard_normal((300, 40, 2))
    S = fa.jl_tensor(Sh, torch.float32)
    out = fa.fused_softmax_(S, S, dims)
    torch.cuda.synchronize()
    assert out.data_ptr() == S.data_ptr()
    assert_close(_np(S), O.fused_softmax(Sh, dims), "float32", "P")


def test_softmax_special_values(fa):
    """-Inf entries give 0; an all -Inf column or a +Inf entry gives NaN, as the
    reference's s .- maximum(s) does."""
    S = np.array([[-np.inf, 0.0, 1.0, 2.0], [-np.inf] * 4, [0.0, np.inf, 1.0, 0.0]]).T   # (4, 3)
    for dtype in DT:
        P = _np(fa.fused_softmax(fa.jl_tensor(S, DT[dtype]), 1))
        ref = O.fused_softmax(S, 1)
        assert np.array_equal(np.isnan(P), np.isnan(ref))
        assert P[0, 0] == 0.0 and abs(P[:, 0].sum() - 1) < 1e-2


def test_softmax_full_size_rows_sum_to_one(fa):
    """A 4096×4096×64 bf16 score tensor (configs[1]'s S per slab) along both dims."""
    g = torch.Generator(device="cuda").manual_seed(3)
    S = fa.jl_empty((4096, 4096, 8), torch.bfloat16)
    S.copy_(torch.randn((4096, 4096, 8), generator=g, device="cuda") * 3)
    for dims in (1, 2):
        P = fa.fused_softmax(S, dims)
        torch.cuda.synchronize()
        sums = P.float().sum(dim=dims - 1)
        assert torch.allclose(sums, torch.ones_like(sums), atol=2e-2)
        ref = torch.softmax(S[:, :, :1].float(), dim=dims - 1)
        assert torch.allclose(P[:, :, :1].float(), ref, atol=2e-2 * ref.abs().max().item() + 1e-3)
