"""GPU parity of the hand-scheduled forward (fa2_fwd_hs_kernel, r05) against the oracle.

The kernel runs the generated inline-asm tile loop (cuda-flash-attention_amd/gen/
gen_fwd_hs.py) for D = 64 and 128 on whole 64-key tiles: two 32-row query chains per
wave, one wave per SIMD.  It is the library's default forward wherever its grid holds at
least one 256-row workgroup per CU (C3, C4, C5, the S = 4096 sweep point); FWD_HS = 1
forces it onto smaller grids here so that every path is reachable at oracle-sized
shapes: one and several 256-row blocks per head, a last block with rows past S, the
restart path (a late score spike), N(0,1) data, both tile types.  Tolerances are the
north star's (fp16 tiles 1e-2 on O and LSE; bf16, the extension, 2e-2).
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

import fa2amd  # noqa: E402
from oracle import fa2_oracle as fo  # noqa: E402

pytestmark = pytest.mark.gpu
TOL = {"fp16": 1e-2, "bf16": 2e-2}


def cuda(*xs):
    return [torch.from_numpy(np.ascontiguousarray(x)).cuda() for x in xs]


def maxerr(a, b):
    return float(np.abs(np.asarray(a, np.float64) - np.asarray(b, np.float64)).max())


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    fa2amd.lib()


@pytest.fixture(autouse=True)
def _no_overrides():
    fa2amd.tune_set(None)
    yield
    fa2amd.tune_set(None)


def run(q, k, v, precision, hs=1):
    fa2amd.tune_set("FWD_HS", hs)
    tq, tk, tv = cuda(q, k, v)
    o, lse = fa2amd.forward(tq, tk, tv, precision)
    torch.cuda.synchronize()
    return o.cpu().numpy(), lse.cpu().numpy()


# S: the two-tile minimum, odd tile counts (the loop's two-tile unroll ends in its middle),
# a last block with rows past S (S % 256 != 0), several blocks per head
HS_SHAPES = [(1, 1, 128, 64), (1, 2, 192, 64), (2, 1, 256, 64), (1, 2, 320, 64), (1, 3, 832, 64),
             (1, 1, 2048, 64), (1, 1, 128, 128), (1, 2, 192, 128), (2, 1, 448, 128), (1, 1, 1024, 128)]


@pytest.mark.parametrize("precision", ["fp16", "bf16"])
@pytest.mark.parametrize("shape", HS_SHAPES, ids=lambda s: "B%d_H%d_S%d_D%d" % s)
def test_hs_forward_vs_oracle(shape, precision):
    B, H, S, D = shape
    q, k, v = fo.harness_inputs(B, H, S, D)
    eo, el = fo.attention_forward(q, k, v)
    o, lse = run(q, k, v, precision, hs=1)
    assert np.isfinite(o).all() and np.isfinite(lse).all()
    assert maxerr(o, eo) < TOL[precision]
    assert maxerr(lse, el) < TOL[precision]


@pytest.mark.parametrize("precision", ["fp16", "bf16"])
@pytest.mark.parametrize("D", [64, 128])
def test_hs_forward_gaussian(D, precision):
    """N(0,1) Q, K, V (the CLI's generator): negative values and larger score spread"""
    q, k, v = fo.cli_inputs(2, 2, 512, D, seed=11)
    eo, el = fo.attention_forward(q, k, v)
    o, lse = run(q, k, v, precision, hs=1)
    assert maxerr(o, eo) < TOL[precision]
    assert maxerr(lse, el) < TOL[precision]


@pytest.mark.parametrize("precision", ["fp16", "bf16"])
@pytest.mark.parametrize("D", [64, 128])
@pytest.mark.parametrize("where", [70, 500], ids=["mid", "late"])
def test_hs_forward_restart(D, precision, where):
    """A key whose scores jump far above the first tile's row max: the tile-sum guard
    flags the block and the robust loop recomputes it (both chains of every wave)."""
    B, H, S = 1, 2, 576
    q, k, v = fo.harness_inputs(B, H, S, D)
    k = k.copy()
    k[:, :, where, :] = 3.0
    eo, el = fo.attention_forward(q, k, v)
    o, lse = run(q, k, v, precision, hs=1)
    assert maxerr(o, eo) < TOL[precision]
    assert maxerr(lse, el) < TOL[precision]


@pytest.mark.parametrize("D", [64, 128])
def test_hs_forward_deterministic(D):
    q, k, v = fo.harness_inputs(1, 4, 1024, D, seed=5)
    o1, l1 = run(q, k, v, "fp16", hs=1)
    o2, l2 = run(q, k, v, "fp16", hs=1)
    assert np.array_equal(o1, o2) and np.array_equal(l1, l2)


@pytest.mark.parametrize("D", [64, 128])
def test_hs_matches_previous_kernel(D):
    """FWD_HS = 0 runs the compiler-scheduled 8-wave kernel on the same inputs: both hold
    the oracle's tolerance, and they agree with each other far inside it."""
    q, k, v = fo.harness_inputs(2, 4, 1024, D, seed=9)
    o1, l1 = run(q, k, v, "fp16", hs=1)
    o0, l0 = run(q, k, v, "fp16", hs=0)
    assert maxerr(o1, o0) < 2e-3
    assert maxerr(l1, l0) < 2e-3


def test_hs_is_default_on_full_grids():
    """C3's grid (512 workgroups of 256 rows) takes the hand-scheduled kernel by default:
    the default and the forced result are bitwise equal, the FWD_HS = 0 result is not."""
    q, k, v = fo.harness_inputs(4, 16, 2048, 64, seed=1)
    od, ld = run(q, k, v, "fp16", hs=-1)
    of, lf = run(q, k, v, "fp16", hs=1)
    assert np.array_equal(od, of) and np.array_equal(ld, lf)
    eo, el = fo.attention_forward(q[:1, :2], k[:1, :2], v[:1, :2])
    assert maxerr(od[:1, :2], eo) < TOL["fp16"]
    assert maxerr(ld[:1, :2], el) < TOL["fp16"]


@pytest.mark.parametrize("shape", [(1, 1, 100, 64), (1, 1, 64, 64), (1, 1, 256, 32)])
def test_hs_forced_on_unserved_shape_is_an_error(shape):
    """FWD_HS = 1 where the kernel cannot serve (ragged S, S < 128, D = 32, which has no
    hand-scheduled kernel) is an error, never a silent launch of another plan"""
    fa2amd.tune_set("FWD_HS", 1)
    q, k, v = cuda(*fo.harness_inputs(*shape))
    with pytest.raises(fa2amd.FA2Error):
        fa2amd.forward(q, k, v, "fp16")


@pytest.mark.parametrize("other", [("FWD_WAVES", 8), ("FWD_KS", 2), ("FWD_NKB", 2)])
def test_hs_forced_with_other_plan_knobs_is_an_error(other):
    fa2amd.tune_set("FWD_HS", 1)
    fa2amd.tune_set(*other)
    q, k, v = cuda(*fo.harness_inputs(1, 2, 512, 64))
    with pytest.raises(fa2amd.FA2Error):
        fa2amd.forward(q, k, v, "fp16")


@pytest.mark.parametrize("D", [64, 128])
def test_hs_forward_restart_some_waves(D):
    """A late key that spikes the scores of ONE wave's 64 rows only (query rows 64..127 of
    the first block get a large first component, the late key too: +15 nats, past the
    2^13 tile-sum guard, for those rows only): that wave recomputes with the rescaling
    loop, the other waves keep their loop results; every row matches the oracle.  (fp16
    tiles: at scores of ~20 nats bf16's 8-bit significand alone is worth ~0.03 in LSE)"""
    B, H, S = 1, 2, 1024
    q, k, v = fo.harness_inputs(B, H, S, D, seed=13)
    q, k = q.copy(), k.copy()
    q[:, :, 64:128, 0] = 10.0
    k[:, :, 900, 0] = 12.0 * np.sqrt(D / 64.0)
    eo, el = fo.attention_forward(q, k, v)
    o, lse = run(q, k, v, "fp16", hs=1)
    assert np.isfinite(o).all() and np.isfinite(lse).all()
    assert maxerr(o, eo) < TOL["fp16"]
    assert maxerr(lse, el) < TOL["fp16"]
