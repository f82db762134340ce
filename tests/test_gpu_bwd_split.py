"""GPU parity of the split backward (BWD_SPLIT, r06) against the oracle.

On grids below one 256-row workgroup per CU the split backward runs the hand-scheduled
dQ kernel on P key chunks per head (Δ fused, written by chunk 0) and the hand-scheduled
dK/dV kernel on P query chunks, both leaving fp32 parts in the stream's scratch block,
then one reduce sums the parts in chunk order (deterministic).  BWD_SPLIT = P forces it
at oracle-sized shapes: several chunk counts including 3, rows past S in the last block,
every exit of the dK/dV loop's three-step unroll (chunks of 2..6 steps), N(0,1) inputs,
both tile types, the forward split before it in one graph capture.  Tolerances: the
north star's (1e-2 fp16, 2e-2 bf16, gradients scaled by max(1, max|ref|)).
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


def _case(shape, seed=3, gauss=False):
    B, H, S, D = shape
    q, k, v = (fo.cli_inputs if gauss else fo.harness_inputs)(B, H, S, D, seed=seed)
    do = np.random.RandomState(seed + 1).randn(B, H, S, D).astype(np.float32)
    eo, el = fo.attention_forward(q, k, v)
    edq, edk, edv, edl = fo.attention_backward(q, k, v, do)
    return (q, k, v, do, eo.astype(np.float32), el.astype(np.float32)), (edq, edk, edv, edl)


def run(inputs, precision, split=None, **knobs):
    if split is not None:
        fa2amd.tune_set("BWD_SPLIT", split)
    for kk, vv in knobs.items():
        fa2amd.tune_set(kk, vv)
    tq, tk, tv, tdo, to, tl = cuda(*inputs)
    dl = torch.empty_like(tl)
    dq, dk, dv = fa2amd.backward(tq, tk, tv, to, tdo, tl, precision, delta_buf=dl)
    torch.cuda.synchronize()
    return [t.cpu().numpy() for t in (dq, dk, dv, dl)]


def check(got, exp, precision):
    for g, e in zip(got[:3], exp[:3]):
        assert np.isfinite(g).all()
        assert maxerr(g, e) < TOL[precision] * max(1.0, float(np.abs(e).max()))
    assert maxerr(got[3], exp[3]) < 1e-4 * max(1.0, float(np.abs(exp[3]).max()))


# (shape, P): chunks of 2 .. 6 64-row steps (every exit of the dK/dV loop's unroll of 3),
# 3 chunks and rows past S (576 = 2.25 blocks of 256), several blocks per head
CASES = [((1, 2, 1024, 64), 2), ((1, 2, 1024, 64), 4), ((1, 2, 1024, 64), 8), ((2, 1, 768, 64), 3),
         ((1, 2, 576, 64), 3), ((1, 1, 1280, 64), 4), ((1, 3, 512, 64), 2), ((2, 2, 1536, 64), 6)]


@pytest.mark.parametrize("precision", ["fp16", "bf16"])
@pytest.mark.parametrize("shape,P", CASES, ids=lambda x: "B%d_H%d_S%d_D%d" % x if isinstance(x, tuple) else f"P{x}")
def test_split_backward_vs_oracle(shape, P, precision):
    inputs, exp = _case(shape)
    check(run(inputs, precision, split=P), exp, precision)


def test_split_backward_gaussian():
    inputs, exp = _case((1, 2, 1024, 64), seed=11, gauss=True)
    check(run(inputs, "fp16", split=4), exp, "fp16")


@pytest.mark.parametrize("P", [2, 4])
def test_split_backward_deterministic(P):
    inputs, _ = _case((1, 2, 2048, 64), seed=5)
    a = run(inputs, "fp16", split=P)
    b = run(inputs, "fp16", split=P)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)


def test_split_backward_matches_unsplit():
    """the split and the hand-scheduled two-kernel plan agree far inside the tolerance"""
    inputs, _ = _case((1, 4, 2048, 64), seed=9)
    a = run(inputs, "fp16", split=4)
    fa2amd.tune_set(None)
    b = run(inputs, "fp16", BWD_SPLIT=1, BWD_FUSED=0, DQ_HS=1, DKDV_HS=1)
    for x, y in zip(a, b):
        assert maxerr(x, y) < 2e-3 * max(1.0, float(np.abs(y).max()))


def auto_split(bh, S, D):
    """the library's rule (f-attn2-backward_f16.cu, bwd_split_auto)"""
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    g = bh * ((S + 255) // 256)
    if D != 64 or g >= ncu or S % 64 or not ((S >= 4096 and g <= 64) or (S >= 2048 and g <= 16)):
        return 1
    P = 1
    while P < 8 and g * 2 * P <= ncu and S % (128 * P) == 0 and S // (2 * P) >= 256:
        P *= 2
    return P


@pytest.mark.parametrize("shape", [(1, 2, 4096, 64), (1, 8, 4096, 64), (1, 2, 2048, 64), (1, 4, 2048, 64),
                                   (2, 4, 1024, 64)])
def test_split_backward_auto_rule(shape):
    """the default plan is the split with bwd_split_auto's chunk count where it gives one
    (bitwise equal to forcing it), and holds the tolerance either way"""
    B, H, S, D = shape
    inputs, _ = _case(shape, seed=2)
    d = run(inputs, "fp16")
    P = auto_split(B * H, S, D)
    if P > 1:
        f = run(inputs, "fp16", split=P)
        for x, y in zip(d, f):
            assert np.array_equal(x, y)
    q, k, v, do = (x[:1, :1] for x in inputs[:4])
    edq, edk, edv, _ = fo.attention_backward(q, k, v, do)
    for g, e in zip(d[:3], (edq, edk, edv)):
        assert maxerr(g[:1, :1], e) < TOL["fp16"] * max(1.0, float(np.abs(e).max()))


@pytest.mark.parametrize("shape,P", [((1, 1, 1000, 64), 2), ((1, 1, 512, 64), 8), ((1, 1, 768, 64), 5),
                                     ((1, 1, 1024, 32), 2), ((1, 1, 1024, 128), 2)],
                         ids=["ragged", "chunk_below_128", "chunk_not_steps", "D32", "D128"])
def test_split_backward_forced_on_unserved_shape_is_an_error(shape, P):
    fa2amd.tune_set("BWD_SPLIT", P)
    B, H, S, D = shape
    tq, tk, tv, tdo = cuda(*fo.harness_inputs(B, H, S, D), np.ones((B, H, S, D), np.float32))
    o, lse = fa2amd.forward(tq, tk, tv, "fp16")
    with pytest.raises(fa2amd.FA2Error):
        fa2amd.backward(tq, tk, tv, o, tdo, lse, "fp16")


@pytest.mark.parametrize("other", [("BWD_FUSED", 0), ("BWD_FUSED", 1), ("DQ_HS", 1), ("DKDV_HS", 0), ("DQ_KS", 2),
                                   ("DKDV_QS", 2), ("BWD_SPLIT", -1)])
def test_split_backward_forced_with_conflicting_knobs_is_an_error(other):
    tq, tk, tv, tdo = cuda(*fo.harness_inputs(1, 2, 1024, 64), np.ones((1, 2, 1024, 64), np.float32))
    o, lse = fa2amd.forward(tq, tk, tv, "fp16")
    fa2amd.tune_set("BWD_SPLIT", 2)
    fa2amd.tune_set(*other)
    with pytest.raises(fa2amd.FA2Error):
        fa2amd.backward(tq, tk, tv, o, tdo, lse, "fp16")


def test_split_step_graph_capture():
    """forward and backward split in one captured step: the capture takes the warm-up's
    block for the forward and reuses it for the backward; replays are bitwise the eager
    step"""
    B, H, S, D = 1, 2, 4096, 64
    fa2amd.tune_set("FWD_SPLIT", 4)
    fa2amd.tune_set("BWD_SPLIT", 4)
    q, k, v = fo.cli_inputs(B, H, S, D, seed=21)
    do = np.random.RandomState(22).randn(B, H, S, D).astype(np.float32)
    tq, tk, tv, tdo = cuda(q, k, v, do)
    o, lse = torch.empty_like(tq), torch.empty(B, H, S, device=tq.device)
    dq, dk, dv = torch.empty_like(tq), torch.empty_like(tq), torch.empty_like(tq)
    dl = torch.empty(B, H, S, device=tq.device)

    def step():
        fa2amd.forward(tq, tk, tv, "fp16", out=o, lse=lse)
        fa2amd.backward(tq, tk, tv, o, tdo, lse, "fp16", dq=dq, dk=dk, dv=dv, delta_buf=dl)

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        step()
        torch.cuda.synchronize()
        eager = [t.clone() for t in (o, lse, dq, dk, dv)]
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=side):
            step()
    torch.cuda.current_stream().wait_stream(side)
    for _ in range(2):
        for t in (o, lse, dq, dk, dv):
            t.fill_(float("nan"))
        graph.replay()
        torch.cuda.synchronize()
        for name, a, b in zip(("o", "lse", "dq", "dk", "dv"), eager, (o, lse, dq, dk, dv)):
            assert torch.equal(a, b), name


def test_split_plans_on_two_streams_at_once():
    """two streams run split forward + backward steps concurrently: each stream has its own
    scratch block, so both give bitwise what a lone step gives"""
    fa2amd.tune_set("FWD_SPLIT", 4)
    fa2amd.tune_set("BWD_SPLIT", 4)
    cases = []
    for seed in (31, 32):
        (q, k, v, do, _, _), _ = _case((1, 2, 2048, 64), seed=seed)
        tq, tk, tv, tdo = cuda(q, k, v, do)
        cases.append((tq, tk, tv, tdo))

    def step(tq, tk, tv, tdo):
        o, lse = fa2amd.forward(tq, tk, tv, "fp16")
        return (o, lse) + tuple(fa2amd.backward(tq, tk, tv, o, tdo, lse, "fp16"))

    alone = []
    for c in cases:
        alone.append([t.clone() for t in step(*c)])
        torch.cuda.synchronize()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    for s in streams:
        s.wait_stream(torch.cuda.current_stream())
    outs = [None, None]
    for _ in range(3):
        for i, (s, c) in enumerate(zip(streams, cases)):
            with torch.cuda.stream(s):
                outs[i] = step(*c)
        torch.cuda.synchronize()
        for a, b in zip(alone, outs):
            for x, y in zip(a, b):
                assert torch.equal(x, y)


def test_split_long_heads_match_the_unsplit_plans():
    """B1_H2_S8192 (the auto rules split both passes, P = 4): forward and gradients agree
    with the unsplit hand-scheduled plans far inside the tolerance, and the forward with
    the oracle on a sample of rows"""
    B, H, S, D = 1, 2, 8192, 64
    q, k, v = fo.harness_inputs(B, H, S, D, seed=12)
    do = np.random.RandomState(13).randn(B, H, S, D).astype(np.float32)
    tq, tk, tv, tdo = cuda(q, k, v, do)

    def step(**knobs):
        fa2amd.tune_set(None)
        for kk, vv in knobs.items():
            fa2amd.tune_set(kk, vv)
        o, lse = fa2amd.forward(tq, tk, tv, "fp16")
        grads = fa2amd.backward(tq, tk, tv, o, tdo, lse, "fp16")
        torch.cuda.synchronize()
        return [t.cpu().numpy() for t in (o, lse) + tuple(grads)]

    split = step()
    ref = step(FWD_SPLIT=1, FWD_HS=1, BWD_SPLIT=1, BWD_FUSED=0, DQ_HS=1, DKDV_HS=1)
    for a, b in zip(split, ref):
        assert maxerr(a, b) < 2e-3 * max(1.0, float(np.abs(b).max()))
    rows = np.arange(0, S, 509)
    s = (q[0, 0, rows].astype(np.float64) @ k[0, 0].astype(np.float64).T) / np.sqrt(D)
    m = s.max(axis=1, keepdims=True)
    p = np.exp(s - m)
    eo = (p @ v[0, 0].astype(np.float64)) / p.sum(axis=1, keepdims=True)
    el = (m[:, 0] + np.log(p.sum(axis=1)))
    assert maxerr(split[0][0, 0, rows], eo) < TOL["fp16"]
    assert maxerr(split[1][0, 0, rows], el) < TOL["fp16"]
