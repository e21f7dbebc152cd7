"""The (batch × head) sharding of SURVEY §8e with the HIP kernels doing the work:
every rank's share (fa_hip.shard.local_slabs: a zero-copy view of a contiguous slab
range) goes through fa_dense_fwd / fa_dense_bwd by itself, as one process per GPU
runs it, and the concatenated shares must be BITWISE the full-batch call (slabs are
independent), with slab 0 within the 16-bit tolerance of the float64 oracle.

The ranks run one after another in this process: a multi-process run would have to
start its ranks from a process that has not touched the GPU (bench.py --gpus N does;
a pytest process has), and its process-group plumbing is covered on CPU by
tests/test_dist.py and tests/test_bench_dist.py (gloo, world size 2)."""
from __future__ import annotations

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def fa():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm device")
    import fa_hip
    fa_hip.lib()
    return fa_hip


def _inputs(fa, N, d, BH):
    g = torch.Generator(device="cuda").manual_seed(7)
    mk = lambda: fa.jl_tensor(torch.randn((N, d, BH), generator=g, device="cuda"), torch.bfloat16)
    return mk(), mk(), mk(), mk()


# (1024, 64, 5): split-KV forward and two-pass backward, 3 + 2 slabs; (4096, 64, 64) =
# configs[1] over 2 ranks and 4x its slabs over 8 (32 per rank: no split-KV on either
# side, which would change the rounding): the default forward kernel and the single pass
@pytest.mark.parametrize("shape,world", [((1024, 64, 5), 2), ((4096, 64, 64), 2), ((4096, 64, 256), 8)])
def test_sharded_hip_matches_full_batch(fa, shape, world):
    from fa_hip.shard import local_slabs, shard_range
    from oracle import fa_oracle as O
    N, d, BH = shape
    Q, K, V, dO = _inputs(fa, N, d, BH)
    y, l, m = fa.dense_fa(Q, K, V)
    full = (y, l, m) + tuple(fa.dense_fa_backward(Q, K, V, y, dO, l, m))

    parts = []
    for rank in range(world):
        a, b = shard_range(BH, world, rank)
        lq, lk, lv, ldo = (local_slabs(t, world, rank) for t in (Q, K, V, dO))
        assert lq.data_ptr() == Q.data_ptr() + a * N * d * Q.element_size()   # zero-copy
        ys, ls, ms = fa.dense_fa(lq, lk, lv)
        parts.append((ys, ls, ms) + tuple(fa.dense_fa_backward(lq, lk, lv, ys, ldo, ls, ms)))
        assert parts[-1][0].shape[-1] == b - a
    torch.cuda.synchronize()
    for i, name in enumerate(("y", "l", "m", "dq", "dk", "dv")):
        got = torch.cat([p[i] for p in parts], dim=-1)
        assert torch.equal(got, full[i]), f"{name}: sharded result differs from the full-batch call"

    sl = lambda t: t[:, :, :1].float().cpu().double().numpy()
    yo, lo, mo = O.dense_fa3(sl(Q), sl(K), sl(V))
    assert np.abs(sl(y) - yo).max() <= 2e-2 * (1 + np.abs(yo).max())
    gq, gk, gv = O.dense_fa_backward(sl(Q), sl(K), sl(V), sl(y), sl(dO), l[:, :, :1].cpu().double().numpy(),
                                     m[:, :, :1].cpu().double().numpy())
    for t, ref in zip(full[3:], (gq, gk, gv)):
        assert np.linalg.norm(sl(t) - ref) <= 2e-2 * np.linalg.norm(ref)
