"""GPU parity of the key-chunk split forward (FWD_SPLIT, r06) against the oracle.

Grids below one 256-row workgroup per CU (the north star's sweep sharded over GPUs: 2-8
heads per GPU) leave CUs idle while every workgroup streams its head's whole K/V.  The
split plan runs the hand-scheduled forward on P key chunks of S / P keys per head, each
workgroup leaving an unnormalised partial (O rows, m, l) in a per-stream scratch block,
and a merge pass combines the P partials in chunk order (deterministic).  FWD_SPLIT = P
forces it here at oracle-sized shapes: several chunk counts, a chunk count that is not a
power of two, rows past S in the last query block, the restart path inside a chunk, both
tile types and head dims, graph capture, scratch growth.  Tolerances: the north star's
(fp16 tiles 1e-2, bf16 2e-2).
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


def run(q, k, v, precision, split=None, **knobs):
    if split is not None:
        fa2amd.tune_set("FWD_SPLIT", split)
    for kk, vv in knobs.items():
        fa2amd.tune_set(kk, vv)
    tq, tk, tv = cuda(q, k, v)
    o, lse = fa2amd.forward(tq, tk, tv, precision)
    torch.cuda.synchronize()
    return o.cpu().numpy(), lse.cpu().numpy()


def auto_split(bh, S, D):
    """the library's rule (kernel_fa2_optimized_f16.cu, fwd_split_auto)"""
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    g = bh * ((S + 255) // 256)
    tiny = D == 64 and S >= 2048 and g <= 16
    min_s, min_chunk = (1024, 256) if D == 128 else (4096, 512 if tiny else 1024)
    if g >= ncu or S % 64 or (S < min_s and not tiny):
        return 1
    P = 1
    while P < 4 and g * 2 * P <= ncu and S % (128 * P) == 0 and S // (2 * P) >= min_chunk:
        P *= 2
    return 1 if D == 64 and P < 4 else P


# (shape, P): 2..16 chunks, 3 chunks (576 = 9 tiles; rows past S in the last query block),
# the 128-key minimum chunk, several query blocks per head, D = 128
CASES = [((1, 2, 1024, 64), 2), ((1, 2, 1024, 64), 4), ((1, 2, 1024, 64), 8), ((2, 3, 512, 64), 4),
         ((1, 1, 2048, 64), 16), ((1, 2, 576, 64), 3), ((2, 1, 1536, 64), 6), ((1, 2, 1024, 128), 4),
         ((1, 1, 768, 128), 3)]


@pytest.mark.parametrize("precision", ["fp16", "bf16"])
@pytest.mark.parametrize("shape,P", CASES, ids=lambda x: "B%d_H%d_S%d_D%d" % x if isinstance(x, tuple) else f"P{x}")
def test_split_forward_vs_oracle(shape, P, precision):
    B, H, S, D = shape
    q, k, v = fo.harness_inputs(B, H, S, D)
    eo, el = fo.attention_forward(q, k, v)
    o, lse = run(q, k, v, precision, split=P)
    assert np.isfinite(o).all() and np.isfinite(lse).all()
    assert maxerr(o, eo) < TOL[precision]
    assert maxerr(lse, el) < TOL[precision]


@pytest.mark.parametrize("D", [64, 128])
def test_split_forward_gaussian(D):
    q, k, v = fo.cli_inputs(1, 3, 1024, D, seed=17)
    eo, el = fo.attention_forward(q, k, v)
    o, lse = run(q, k, v, "fp16", split=4)
    assert maxerr(o, eo) < TOL["fp16"]
    assert maxerr(lse, el) < TOL["fp16"]


@pytest.mark.parametrize("D", [64, 128])
@pytest.mark.parametrize("where", [10, 300, 1000], ids=["chunk0", "chunk1", "chunk3"])
def test_split_forward_restart(D, where):
    """a late score spike inside one key chunk: that chunk's workgroups redo their rows with
    the rescaling loop over the chunk and leave its partial; the other chunks do not see
    it; the merge weighs the chunks by their m"""
    q, k, v = fo.harness_inputs(1, 2, 1024, D, seed=3)
    k = k.copy()
    k[:, :, where, :] = 3.0
    eo, el = fo.attention_forward(q, k, v)
    o, lse = run(q, k, v, "fp16", split=4)
    assert maxerr(o, eo) < TOL["fp16"]
    assert maxerr(lse, el) < TOL["fp16"]


def test_split_forward_restart_some_waves():
    """one wave's rows spike in one chunk only (the other waves keep their loop result)"""
    q, k, v = fo.harness_inputs(1, 2, 1024, 64, seed=13)
    q, k = q.copy(), k.copy()
    q[:, :, 64:128, 0] = 10.0
    k[:, :, 900, 0] = 12.0
    eo, el = fo.attention_forward(q, k, v)
    o, lse = run(q, k, v, "fp16", split=2)
    assert maxerr(o, eo) < TOL["fp16"]
    assert maxerr(lse, el) < TOL["fp16"]


@pytest.mark.parametrize("P", [2, 8])
def test_split_forward_deterministic(P):
    q, k, v = fo.harness_inputs(1, 2, 2048, 64, seed=5)
    o1, l1 = run(q, k, v, "fp16", split=P)
    o2, l2 = run(q, k, v, "fp16", split=P)
    assert np.array_equal(o1, o2) and np.array_equal(l1, l2)


def test_split_matches_unsplit():
    q, k, v = fo.harness_inputs(1, 4, 2048, 64, seed=9)
    o1, l1 = run(q, k, v, "fp16", split=8)
    fa2amd.tune_set(None)
    o0, l0 = run(q, k, v, "fp16", split=1, FWD_HS=1)
    assert maxerr(o1, o0) < 2e-3
    assert maxerr(l1, l0) < 2e-3


@pytest.mark.parametrize("shape", [(1, 2, 4096, 64), (1, 8, 4096, 64), (1, 2, 2048, 64), (1, 4, 2048, 64),
                                   (2, 8, 1024, 64),
                                   (1, 2, 2048, 128), (2, 8, 1024, 128), (2, 8, 512, 128)])
def test_split_auto_rule(shape):
    """below a full grid the default plan is the split with fwd_split_auto's chunk count
    (bitwise equal to forcing that count), or the unsplit small-grid plans where it gives 1"""
    B, H, S, D = shape
    q, k, v = fo.harness_inputs(B, H, S, D, seed=2)
    od, ld = run(q, k, v, "fp16")
    P = auto_split(B * H, S, D)
    if P > 1:
        of, lf = run(q, k, v, "fp16", split=P)
        assert np.array_equal(od, of) and np.array_equal(ld, lf)
    eo, el = fo.attention_forward(q[:1, :1], k[:1, :1], v[:1, :1])
    assert maxerr(od[:1, :1], eo) < TOL["fp16"]
    assert maxerr(ld[:1, :1], el) < TOL["fp16"]


def test_split_disabled_is_the_small_grid_plan():
    """FWD_SPLIT = 1 restores the unsplit small-grid plan; both hold the tolerance"""
    q, k, v = fo.harness_inputs(1, 2, 2048, 64, seed=4)
    eo, el = fo.attention_forward(q, k, v)
    o1, l1 = run(q, k, v, "fp16", split=1)
    assert maxerr(o1, eo) < TOL["fp16"] and maxerr(l1, el) < TOL["fp16"]


@pytest.mark.parametrize("shape,P", [((1, 1, 1000, 64), 2), ((1, 1, 512, 64), 8), ((1, 1, 768, 64), 5),
                                     ((1, 1, 1024, 32), 2)],
                         ids=["ragged", "chunk_below_128", "chunk_not_tiles", "D32"])
def test_split_forced_on_unserved_shape_is_an_error(shape, P):
    fa2amd.tune_set("FWD_SPLIT", P)
    q, k, v = cuda(*fo.harness_inputs(*shape))
    with pytest.raises(fa2amd.FA2Error):
        fa2amd.forward(q, k, v, "fp16")


@pytest.mark.parametrize("other", [("FWD_HS", 0), ("FWD_WAVES", 8), ("FWD_KS", 2), ("FWD_SPLIT", -1)])
def test_split_forced_with_conflicting_knobs_is_an_error(other):
    fa2amd.tune_set("FWD_SPLIT", 2)
    fa2amd.tune_set(*other)
    q, k, v = cuda(*fo.harness_inputs(1, 2, 1024, 64))
    with pytest.raises(fa2amd.FA2Error):
        fa2amd.forward(q, k, v, "fp16")


def test_split_scratch_grows():
    """a larger split after a smaller one on the same stream grows the block (the stream is
    drained first); both results hold the tolerance"""
    for shape, P in (((1, 1, 512, 64), 2), ((1, 4, 2048, 64), 8), ((1, 2, 1024, 64), 4)):
        q, k, v = fo.harness_inputs(*shape, seed=7)
        eo, el = fo.attention_forward(q, k, v)
        o, lse = run(q, k, v, "fp16", split=P)
        assert maxerr(o, eo) < TOL["fp16"] and maxerr(lse, el) < TOL["fp16"]


def test_split_graph_capture():
    """a capture takes the stream's scratch block from the warm-up call: the replays give
    bitwise the eager result; a capture with no block before it runs the unsplit plan and
    still holds the tolerance"""
    q, k, v = fo.harness_inputs(1, 2, 2048, 64, seed=8)
    eo, el = fo.attention_forward(q, k, v)
    tq, tk, tv = cuda(q, k, v)
    o, lse = torch.empty_like(tq), torch.empty(1, 2, 2048, device=tq.device)
    for warm in (True, False):
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            if warm:
                fa2amd.forward(tq, tk, tv, "fp16", out=o, lse=lse)
                torch.cuda.synchronize()
                ref = (o.clone(), lse.clone())
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph, stream=side):
                fa2amd.forward(tq, tk, tv, "fp16", out=o, lse=lse)
        torch.cuda.current_stream().wait_stream(side)
        for _ in range(2):
            o.fill_(float("nan"))
            graph.replay()
            torch.cuda.synchronize()
            if warm:
                assert torch.equal(o, ref[0]) and torch.equal(lse, ref[1])
            assert maxerr(o.cpu().numpy(), eo) < TOL["fp16"]
            assert maxerr(lse.cpu().numpy(), el) < TOL["fp16"]


def test_host_release_frees_scratch_and_next_call_reallocates():
    q, k, v = fo.harness_inputs(1, 2, 1024, 64, seed=6)
    o1, l1 = run(q, k, v, "fp16", split=4)
    fa2amd.host_release()
    o2, l2 = run(q, k, v, "fp16", split=4)
    assert np.array_equal(o1, o2) and np.array_equal(l1, l2)
