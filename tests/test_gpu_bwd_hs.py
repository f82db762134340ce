"""GPU parity of the hand-scheduled backward kernels (r05) against the oracle.

fa2_bwd_dq_hs_kernel<64> (generated asm loop, gen/gen_bwd_dq.py) computes dQ (and Δ, when
it gets O) and fa2_bwd_dkdv_hs_kernel<64> (gen/gen_bwd_dkdv.py) dK and dV, for D = 64 on
whole 64-row tiles.  Both are the default launches wherever their grid holds at least
one 256-row workgroup per CU (C3, C5, the S = 4096 sweep point).  DQ_HS = 1 /
DKDV_HS = 1 force them onto the small shapes here: one and several 256-row blocks per head, a last block
with rows past S, every exit of the dK/dV loop's three-step unroll, N(0,1) inputs and
gradients, both tile types, Δ fused (O given) and Δ supplied.  Tolerances are the north star's (1e-2 fp16, 2e-2 bf16, gradients scaled
by max(1, max|ref|) as in test_gpu_parity.py).
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


DQ_SHAPES = [(1, 1, 128, 64), (1, 2, 192, 64), (2, 1, 256, 64), (1, 2, 320, 64), (1, 3, 832, 64), (1, 1, 2048, 64)]


def _case(shape, seed=3, gauss=False):
    B, H, S, D = shape
    q, k, v = (fo.cli_inputs if gauss else fo.harness_inputs)(B, H, S, D, seed=seed)
    do = np.random.RandomState(seed + 1).randn(B, H, S, D).astype(np.float32)
    eo, el = fo.attention_forward(q, k, v)
    edq, edk, edv, edl = fo.attention_backward(q, k, v, do)
    return (q, k, v, do, eo.astype(np.float32), el.astype(np.float32)), (edq, edk, edv, edl)


HS_KNOBS = [{"DQ_HS": 1, "DKDV_HS": 0}, {"DQ_HS": 0, "DKDV_HS": 1}, {"DQ_HS": 1, "DKDV_HS": 1}]


@pytest.mark.parametrize("precision", ["fp16", "bf16"])
@pytest.mark.parametrize("knobs", HS_KNOBS, ids=["dq_hs", "dkdv_hs", "both_hs"])
@pytest.mark.parametrize("shape", DQ_SHAPES + [(1, 1, 384, 64), (1, 1, 448, 64)], ids=lambda s: "B%d_H%d_S%d_D%d" % s)
def test_hs_full_backward(shape, knobs, precision):
    """fa2_backward's two-kernel plan with the hand-scheduled dQ (Δ fused, written out for
    dK/dV) and / or the hand-scheduled dK/dV"""
    for key, val in knobs.items():
        fa2amd.tune_set(key, val)
    fa2amd.tune_set("BWD_FUSED", 0)
    (q, k, v, do, o, lse), (edq, edk, edv, _) = _case(shape)
    tq, tk, tv, tdo, to, tl = cuda(q, k, v, do, o, lse)
    dq, dk, dv = fa2amd.backward(tq, tk, tv, to, tdo, tl, precision)
    torch.cuda.synchronize()
    for got, exp in ((dq, edq), (dk, edk), (dv, edv)):
        g = got.cpu().numpy()
        assert np.isfinite(g).all()
        assert maxerr(g, exp) < TOL[precision] * max(1.0, float(np.abs(exp).max()))


@pytest.mark.parametrize("fused_delta", [True, False], ids=["delta_fused", "delta_given"])
@pytest.mark.parametrize("shape", [(1, 2, 320, 64), (2, 2, 1024, 64)], ids=lambda s: "B%d_H%d_S%d_D%d" % s)
def test_hs_dq_entry_points(shape, fused_delta):
    """fa2_backward_dq_delta (Δ from the staged O rows, written out) and fa2_backward_dq (Δ read)"""
    fa2amd.tune_set("DQ_HS", 1)
    (q, k, v, do, o, lse), (edq, _, _, edl) = _case(shape, seed=7, gauss=True)
    tq, tk, tv, tdo, to, tl = cuda(q, k, v, do, o, lse)
    dq = torch.empty_like(tq)
    if fused_delta:
        dl = torch.full(tl.shape, float("nan"), device=tq.device)
        fa2amd.backward_dq_delta(tq, tk, tv, to, tdo, tl, dl, dq)
    else:
        dl = fa2amd.delta(tdo, to)
        fa2amd.backward_dq(tq, tk, tv, tdo, tl, dl, dq)
    torch.cuda.synchronize()
    assert maxerr(dl.cpu().numpy(), edl) < 1e-4 * max(1.0, float(np.abs(edl).max()))
    assert maxerr(dq.cpu().numpy(), edq) < TOL["fp16"] * max(1.0, float(np.abs(edq).max()))


def test_hs_dkdv_entry_point():
    """fa2_backward_dkdv (Δ supplied) through the hand-scheduled kernel"""
    fa2amd.tune_set("DKDV_HS", 1)
    (q, k, v, do, o, lse), (_, edk, edv, edl) = _case((2, 2, 1024, 64), seed=5, gauss=True)
    tq, tk, tv, tdo, to, tl = cuda(q, k, v, do, o, lse)
    dl = fa2amd.delta(tdo, to)
    dk, dv = torch.empty_like(tq), torch.empty_like(tq)
    fa2amd.backward_dkdv(tq, tk, tv, tdo, tl, dl, dk, dv)
    torch.cuda.synchronize()
    for got, exp in ((dk, edk), (dv, edv)):
        assert maxerr(got.cpu().numpy(), exp) < TOL["fp16"] * max(1.0, float(np.abs(exp).max()))


def test_hs_dkdv_deterministic_and_default():
    """bitwise repeatable; at C3's grid the default dK/dV launch is the hand-scheduled one"""
    B, H, S, D = 4, 16, 2048, 64
    q, k, v = fo.harness_inputs(B, H, S, D, seed=4)
    do = np.random.RandomState(10).randn(B, H, S, D).astype(np.float32)
    tq, tk, tv, tdo = cuda(q, k, v, do)
    o, lse = fa2amd.forward(tq, tk, tv, "fp16")
    res = []
    for hs in (-1, 1, 1, 0):
        fa2amd.tune_set("DKDV_HS", hs)
        dq, dk, dv = fa2amd.backward(tq, tk, tv, o, tdo, lse, "fp16")
        torch.cuda.synchronize()
        res.append((dk.cpu().numpy(), dv.cpu().numpy()))
    for t in range(2):
        assert np.array_equal(res[0][t], res[1][t]) and np.array_equal(res[1][t], res[2][t])
        assert maxerr(res[1][t], res[3][t]) < 2e-3 * max(1.0, float(np.abs(res[3][t]).max()))
    _, edk, edv, _ = fo.attention_backward(q[:1, :2], k[:1, :2], v[:1, :2], do[:1, :2])
    assert maxerr(res[1][0][:1, :2], edk) < TOL["fp16"] * max(1.0, float(np.abs(edk).max()))
    assert maxerr(res[1][1][:1, :2], edv) < TOL["fp16"] * max(1.0, float(np.abs(edv).max()))


def test_hs_dq_deterministic_and_default():
    """bitwise repeatable; at C3's grid the default dQ launch is the hand-scheduled one"""
    B, H, S, D = 4, 16, 2048, 64
    q, k, v = fo.harness_inputs(B, H, S, D, seed=2)
    do = np.random.RandomState(9).randn(B, H, S, D).astype(np.float32)
    tq, tk, tv, tdo = cuda(q, k, v, do)
    o, lse = fa2amd.forward(tq, tk, tv, "fp16")
    res = []
    for hs in (-1, 1, 1, 0):
        fa2amd.tune_set("DQ_HS", hs)
        dq, dk, dv = fa2amd.backward(tq, tk, tv, o, tdo, lse, "fp16")
        torch.cuda.synchronize()
        res.append(dq.cpu().numpy())
    assert np.array_equal(res[0], res[1]) and np.array_equal(res[1], res[2])
    assert maxerr(res[1], res[3]) < 2e-3 * max(1.0, float(np.abs(res[3]).max()))
    edq, _, _, _ = fo.attention_backward(q[:1, :2], k[:1, :2], v[:1, :2], do[:1, :2])
    assert maxerr(res[1][:1, :2], edq) < TOL["fp16"] * max(1.0, float(np.abs(edq).max()))


@pytest.mark.parametrize("knob", ["DQ_HS", "DKDV_HS"])
@pytest.mark.parametrize("shape", [(1, 1, 100, 64), (1, 1, 64, 64)])
def test_hs_bwd_forced_on_unserved_shape_is_an_error(shape, knob):
    fa2amd.tune_set(knob, 1)
    fa2amd.tune_set("BWD_FUSED", 0)
    (q, k, v, do, o, lse), _ = _case(shape)
    tq, tk, tv, tdo, to, tl = cuda(q, k, v, do, o, lse)
    with pytest.raises(fa2amd.FA2Error):
        fa2amd.backward(tq, tk, tv, to, tdo, tl, "fp16")


@pytest.mark.parametrize("knob", ["DQ_HS", "DKDV_HS"])
def test_hs_bwd_forced_onto_the_fused_plan_is_an_error(knob):
    """a small grid picks the fused one-launch backward, which has no hand-scheduled
    roles: forcing DQ_HS / DKDV_HS there (without BWD_FUSED = 0) is an error"""
    fa2amd.tune_set(knob, 1)
    (q, k, v, do, o, lse), _ = _case((1, 2, 256, 64))
    tq, tk, tv, tdo, to, tl = cuda(q, k, v, do, o, lse)
    with pytest.raises(fa2amd.FA2Error):
        fa2amd.backward(tq, tk, tv, to, tdo, tl, "fp16")


@pytest.mark.parametrize("knobs", [{"DQ_HS": 1, "DQ_WAVES": 8}, {"DQ_HS": 1, "DQ_KS": 2},
                                   {"DKDV_HS": 1, "DKDV_WAVES": 8}, {"DKDV_HS": 1, "DKDV_QS": 2}],
                         ids=lambda k: "_".join(f"{a}{b}" for a, b in sorted(k.items())))
def test_hs_bwd_forced_with_other_plan_knobs_is_an_error(knobs):
    for key, val in knobs.items():
        fa2amd.tune_set(key, val)
    fa2amd.tune_set("BWD_FUSED", 0)
    (q, k, v, do, o, lse), _ = _case((1, 2, 256, 64))
    tq, tk, tv, tdo, to, tl = cuda(q, k, v, do, o, lse)
    with pytest.raises(fa2amd.FA2Error):
        fa2amd.backward(tq, tk, tv, to, tdo, tl, "fp16")


@pytest.mark.parametrize("knob", ["DQ_HS", "DKDV_HS"])
def test_hs_bwd_forced_at_other_head_dims_is_an_error(knob):
    fa2amd.tune_set(knob, 1)
    fa2amd.tune_set("BWD_FUSED", 0)
    (q, k, v, do, o, lse), _ = _case((1, 2, 256, 32))
    tq, tk, tv, tdo, to, tl = cuda(q, k, v, do, o, lse)
    with pytest.raises(fa2amd.FA2Error):
        fa2amd.backward(tq, tk, tv, to, tdo, tl, "fp16")
