"""GPU parity of the two-chain ping-pong forward (fa2_fwd_pp_kernel, FWD_PP=1)
against the oracle, the way test_gpu_parity.py holds the default forward:
max-abs 1e-2 on O and LSE for fp16 tiles (north star), 2e-2 for bf16.

Shapes cover one tile (S = 1, 33, 64), the peeled first / last iterations at every
parity of the tile count (S = 128, 192, 300, 1000), ragged last tiles, query blocks
past S (partial 256-row workgroups), and the lazy-rescale slow path on both chains
(late high-scoring keys).
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

import fa2amd  # noqa: E402
from oracle import fa2_oracle as fo  # noqa: E402

pytestmark = pytest.mark.gpu

TOL = {"fp16": 1e-2, "bf16": 2e-2}


@pytest.fixture(autouse=True)
def _pp():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    fa2amd.tune_set(None)
    fa2amd.tune_set("FWD_PP", 1)
    yield
    fa2amd.tune_set(None)


def cuda(*xs):
    return [torch.from_numpy(np.ascontiguousarray(x)).cuda() for x in xs]


def maxerr(a, b):
    return float(np.abs(np.asarray(a, np.float64) - np.asarray(b, np.float64)).max())


SHAPES = [(1, 1, 1, 64), (1, 2, 33, 64), (1, 1, 64, 64), (1, 2, 128, 64), (2, 1, 192, 64), (2, 2, 300, 64),
          (1, 1, 1, 128), (1, 2, 129, 128), (2, 1, 1000, 128), (1, 2, 2048, 128),
          (1, 3, 1000, 64), (2, 2, 2048, 64), (1, 1, 4096, 64), (1, 2, 520, 64)]


@pytest.mark.parametrize("precision", ["fp16", "bf16"])
@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "B{}_H{}_S{}_D{}".format(*s))
def test_pp_forward_vs_oracle(shape, precision):
    B, H, S, D = shape
    q, k, v = fo.cli_inputs(B, H, S, D, seed=11)
    eo, el = fo.attention_forward(q, k, v)
    tq, tk, tv = cuda(q, k, v)
    o, lse = fa2amd.forward(tq, tk, tv, precision)
    torch.cuda.synchronize()
    assert np.isfinite(o.cpu().numpy()).all()
    assert maxerr(o.cpu().numpy(), eo) < TOL[precision]
    assert maxerr(lse.cpu().numpy(), el) < TOL[precision]


@pytest.mark.parametrize("shape", [(1, 2, 200, 64), (1, 1, 1000, 64)])
def test_pp_forward_rescale(shape):
    """keys that score far above everything before them, late and mid-sequence, in
    rows of both chains: the guard's slow path (m moves, O and l rescale)"""
    B, H, S, D = shape
    q, k, v = fo.harness_inputs(B, H, S, D)
    k = k.copy()
    k[:, :, S - 3, :] = 3.0
    k[:, :, S // 3, :] = 2.0
    eo, el = fo.attention_forward(q, k, v)
    tq, tk, tv = cuda(q, k, v)
    o, lse = fa2amd.forward(tq, tk, tv, "fp16")
    torch.cuda.synchronize()
    assert maxerr(o.cpu().numpy(), eo) < TOL["fp16"]
    assert maxerr(lse.cpu().numpy(), el) < TOL["fp16"]


def test_pp_matches_default_kernel():
    """same inputs through the default forward: the two kernels agree to fp16-tile
    rounding (they differ only in the order of the row-sum adds)"""
    q, k, v = fo.harness_inputs(2, 4, 777, 64)
    tq, tk, tv = cuda(q, k, v)
    o1, l1 = fa2amd.forward(tq, tk, tv, "fp16")
    fa2amd.tune_set("FWD_PP", 0)
    o0, l0 = fa2amd.forward(tq, tk, tv, "fp16")
    torch.cuda.synchronize()
    assert float((o1 - o0).abs().max()) < 2e-3
    assert float((l1 - l0).abs().max()) < 2e-3


def test_pp_deterministic():
    q, k, v = fo.harness_inputs(2, 2, 1000, 64)
    tq, tk, tv = cuda(q, k, v)
    a = fa2amd.forward(tq, tk, tv, "fp16")
    b = fa2amd.forward(tq, tk, tv, "fp16")
    torch.cuda.synchronize()
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
