"""BASELINE.json's GPU configs at their full sizes, against the C oracle.

The reference harness's pass rule (test_flash_attention2.py:1018-1020, 930-935):
max-abs error over the whole tensor below the tolerance, no NaN/Inf; for the
backward dQ, dK and dV are concatenated before the max, with dO = ones as its
compute_reference_backward draws it (:220-232).  The tolerances are the north
star's, un-scaled: 1e-2 for fp16 tiles (bf16 tiles, an extension, 2e-2).

  C3  B4_H16_S2048_D64   fp16 fwd+bwd   every one of the 64 heads
  C4  B8_H16_S4096_D128  fp16 fwd       every one of the 128 heads; a 4-head bwd at the same S, D
  C5  B64_H16_S2048_D64  fp16 fwd+bwd   one GPU (1024 heads): 158 heads against the oracle
                                        (one whole 8-way shard, 128 heads, and 32 spread over
                                        the tensor), identities on every head; and the
                                        north star's 8-way B*H split through fa2_*_host, every
                                        shard on device 0 (HOST_SHARDS_ON_DEVICE0), so the
                                        non-zero shard offsets of capi.cpp run_shard execute

The checker is oracle/fa2_oracle.c (threaded C restatement of compute_reference and
its closed-form backward, pinned to the reference's golden vectors by
tests/test_oracle_golden.py).  The HIP path is reached only through the C ABI.
"""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

import fa2amd  # noqa: E402
from oracle import c_oracle, fa2_oracle as fo  # noqa: E402

pytestmark = pytest.mark.gpu

TOL = {"fp16": 1e-2, "bf16": 2e-2}


def _threads():
    try:
        n = int(os.environ.get("OMP_NUM_THREADS", "0"))
    except ValueError:
        n = 0
    return max(1, n or min(len(os.sched_getaffinity(0)), 32))


NT = _threads()


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    fa2amd.lib()
    fa2amd.tune_set(None)
    yield
    fa2amd.tune_set(None)


def maxerr(a, b):
    return float(np.abs(np.asarray(a, np.float64) - np.asarray(b, np.float64)).max())


def cuda(*xs):
    return [torch.from_numpy(np.ascontiguousarray(x)).cuda() for x in xs]


def heads(x, idx):
    """rows idx of x viewed as [B*H] heads, as a (1, len(idx), ...) array"""
    flat = x.reshape((-1,) + x.shape[2:])
    return np.ascontiguousarray(flat[idx])[None]


def gpu_fwd_bwd(q, k, v, do, precision):
    tq, tk, tv, tdo = cuda(q, k, v, do)
    o, lse = fa2amd.forward(tq, tk, tv, precision)
    dq, dk, dv = fa2amd.backward(tq, tk, tv, o, tdo, lse, precision)
    torch.cuda.synchronize()
    out = [x.cpu().numpy() for x in (o, lse, dq, dk, dv)]
    del tq, tk, tv, tdo, o, lse, dq, dk, dv
    torch.cuda.empty_cache()
    return out


def assert_identities(q, v, do, o, dk, dv, atol=0.05):
    """size-independent facts of attention, on every head:
    sum_k dV[k] = sum_q dO[q] (rows of P sum to 1), sum_k dK[k] = 0 (rows of dS sum to
    0), min_k V <= O <= max_k V (rows of O are convex combinations of V's rows)"""
    np.testing.assert_allclose(dv.astype(np.float64).sum(2), do.astype(np.float64).sum(2), atol=atol, rtol=1e-3)
    assert np.abs(dk.astype(np.float64).sum(2)).max() < atol
    assert (o >= v.min(2, keepdims=True) - 1e-3).all() and (o <= v.max(2, keepdims=True) + 1e-3).all()


# ---------------------------------------------------------------------------
# C3: every head, the harness rule
# ---------------------------------------------------------------------------
@pytest.fixture(scope="module")
def c3_oracle():
    B, H, S, D = 4, 16, 2048, 64
    q, k, v = fo.harness_inputs(B, H, S, D)
    ones = np.ones_like(q)
    eo, el = c_oracle.forward(q, k, v, NT)
    edq, edk, edv = c_oracle.backward(q, k, v, eo, ones, el, NT)
    return q, k, v, ones, eo, el, np.concatenate([x.ravel() for x in (edq, edk, edv)])


@pytest.mark.parametrize("precision", ["fp16", "bf16"])
def test_c3_every_head_harness_rule(c3_oracle, precision):
    """C3 = B4_H16_S2048_D64 fwd+bwd, harness inputs (seed 42, dO = ones), all 64 heads:
    O, LSE and the concatenated (dQ, dK, dV) within the north star's max-abs bound."""
    q, k, v, ones, eo, el, eg = c3_oracle
    o, lse, dq, dk, dv = gpu_fwd_bwd(q, k, v, ones, precision)
    got = np.concatenate([x.ravel() for x in (dq, dk, dv)])
    for name, a in (("o", o), ("lse", lse), ("grads", got)):
        assert np.isfinite(a).all(), name
    assert maxerr(o, eo) < TOL[precision]
    assert maxerr(lse, el) < TOL[precision]
    assert maxerr(got, eg) < TOL[precision]
    assert_identities(q, v, ones, o, dk, dv)


def randn_do(B, H, S, D):
    """the bench's realistic upstream gradient (bench.py extra_configs.c3_dO_randn):
    dO ~ N(0, 1) from torch.Generator seed 43"""
    return torch.randn(B, H, S, D, generator=torch.Generator().manual_seed(43)).numpy()


@pytest.fixture(scope="module")
def c3_oracle_randn(c3_oracle):
    q, k, v, _, eo, el, _ = c3_oracle
    do = randn_do(4, 16, 2048, 64)
    edq, edk, edv = c_oracle.backward(q, k, v, eo, do, el, NT)
    return do, (edq, edk, edv)


@pytest.mark.parametrize("precision", ["fp16", "bf16"])
def test_c3_every_head_gaussian_gradient(c3_oracle, c3_oracle_randn, precision):
    """C3 fwd+bwd on all 64 heads with dO ~ N(0, 1) (seed 43, the bench's c3_dO_randn
    input) instead of the harness's ones: |dQ| reaches O(1) here (with dO = ones it stays
    below 0.013), so the gradients are held to the tolerance scaled by max(1, max|ref|),
    per tensor, as test_gpu_parity.py does for its N(0, 1) gradients."""
    q, k, v, _, eo, el, _ = c3_oracle
    do, exp = c3_oracle_randn
    o, lse, dq, dk, dv = gpu_fwd_bwd(q, k, v, do, precision)
    assert maxerr(o, eo) < TOL[precision] and maxerr(lse, el) < TOL[precision]
    for got, e in zip((dq, dk, dv), exp):
        assert np.isfinite(got).all()
        assert maxerr(got, e) < TOL[precision] * max(1.0, float(np.abs(e).max()))
    # the column sums of dV are O(100) here: bf16's 8-bit significand is worth ~0.3 on them
    assert_identities(q, v, do, o, dk, dv, atol=0.05 if precision == "fp16" else 0.5)


# ---------------------------------------------------------------------------
# C4: the long-sequence D = 128 forward, every head
# ---------------------------------------------------------------------------
def test_c4_forward_every_head():
    """C4 = B8_H16_S4096_D128 fp16 forward, harness inputs: all 128 heads against the
    oracle (O and LSE, max-abs), and O inside the hull of V on every head."""
    B, H, S, D = 8, 16, 4096, 128
    q, k, v = fo.harness_inputs(B, H, S, D)
    tq, tk, tv = cuda(q, k, v)
    o, lse = fa2amd.forward(tq, tk, tv, "fp16")
    torch.cuda.synchronize()
    o, lse = o.cpu().numpy(), lse.cpu().numpy()
    del tq, tk, tv
    torch.cuda.empty_cache()
    assert np.isfinite(o).all() and np.isfinite(lse).all()
    eo, el = c_oracle.forward(q, k, v, NT)
    assert maxerr(o, eo) < TOL["fp16"]
    assert maxerr(lse, el) < TOL["fp16"]
    assert (o >= v.min(2, keepdims=True) - 1e-3).all() and (o <= v.max(2, keepdims=True) + 1e-3).all()


def test_c4_shape_backward_heads():
    """The backward at C4's S = 4096, D = 128 (4 heads: the D = 128 launch plans), harness
    rule with dO = ones."""
    B, H, S, D = 1, 4, 4096, 128
    q, k, v = fo.harness_inputs(B, H, S, D, seed=44)
    ones = np.ones_like(q)
    o, lse, dq, dk, dv = gpu_fwd_bwd(q, k, v, ones, "fp16")
    eo, el = c_oracle.forward(q, k, v, NT)
    edq, edk, edv = c_oracle.backward(q, k, v, eo, ones, el, NT)
    assert maxerr(o, eo) < TOL["fp16"] and maxerr(lse, el) < TOL["fp16"]
    got = np.concatenate([x.ravel() for x in (dq, dk, dv)])
    assert np.isfinite(got).all()
    assert maxerr(got, np.concatenate([x.ravel() for x in (edq, edk, edv)])) < TOL["fp16"]


# ---------------------------------------------------------------------------
# C5: B64_H16_S2048_D64 on one GPU, and as the north star's 8-way B*H split
# ---------------------------------------------------------------------------
C5 = (64, 16, 2048, 64)
# 158 heads: one whole 8-way shard (heads 640..767, shard 5 of fa2_shard_range) and 32
# heads spread over the tensor, including both ends and every shard's first and last
# head (shards of 128 heads)
C5_SHARD = list(range(5 * 128, 6 * 128))
C5_SAMPLE = sorted({0, 1, 1023} | {s * 128 for s in range(8)} | {s * 128 + 127 for s in range(8)}
                   | {37 + 71 * i for i in range(14)} | set(C5_SHARD))


@pytest.fixture(scope="module")
def c5_data():
    B, H, S, D = C5
    q, k, v = fo.harness_inputs(B, H, S, D)
    ones = np.ones_like(q)
    qs, ks, vs = (heads(x, C5_SAMPLE) for x in (q, k, v))
    eo, el = c_oracle.forward(qs, ks, vs, NT)
    edq, edk, edv = c_oracle.backward(qs, ks, vs, eo, np.ones_like(qs), el, NT)
    return q, k, v, ones, (eo, el, edq, edk, edv)


def _check_c5(c5_data, o, lse, dq, dk, dv):
    q, k, v, ones, (eo, el, edq, edk, edv) = c5_data
    for name, a in (("o", o), ("lse", lse), ("dq", dq), ("dk", dk), ("dv", dv)):
        assert np.isfinite(a).all(), name
    assert maxerr(heads(o, C5_SAMPLE), eo) < TOL["fp16"]
    assert maxerr(heads(lse, C5_SAMPLE), el) < TOL["fp16"]
    got = np.concatenate([heads(x, C5_SAMPLE).ravel() for x in (dq, dk, dv)])
    assert maxerr(got, np.concatenate([x.ravel() for x in (edq, edk, edv)])) < TOL["fp16"]
    assert_identities(q, v, ones, o, dk, dv)


def test_c5_one_gpu(c5_data):
    """C5 fwd+bwd through the device-pointer C ABI on one GPU (the 1-GPU point of the
    north star's scaling curve)."""
    q, k, v, ones, _ = c5_data
    o, lse, dq, dk, dv = gpu_fwd_bwd(q, k, v, ones, "fp16")
    _check_c5(c5_data, o, lse, dq, dk, dv)


def test_c5_host_api_8way_split(c5_data):
    """C5 through fa2_forward_host / fa2_backward_host with num_devices = 8: eight
    contiguous 128-head shards (fa2_shard_range), each copied in, computed and copied
    back by its own host thread; all on device 0 here (HOST_SHARDS_ON_DEVICE0)."""
    q, k, v, ones, _ = c5_data
    fa2amd.tune_set("HOST_SHARDS_ON_DEVICE0", 1)
    try:
        o, lse, ms_f = fa2amd.forward_host(q, k, v, "fp16", num_devices=8)
        dq, dk, dv, ms_b = fa2amd.backward_host(q, k, v, o, ones, lse, "fp16", num_devices=8)
    finally:
        fa2amd.tune_set(None)
    assert ms_f > 0 and ms_b > 0
    _check_c5(c5_data, o, lse, dq, dk, dv)
    # every shard equals the same heads computed as one 128-head problem on the device API
    first, n = fa2amd.shard_range(1024, 8, 5)
    sl = list(range(first, first + n))
    o1, l1, dq1, dk1, dv1 = gpu_fwd_bwd(heads(q, sl), heads(k, sl), heads(v, sl), heads(ones, sl), "fp16")
    for a, b in ((o, o1), (lse, l1), (dq, dq1), (dk, dk1), (dv, dv1)):
        assert np.array_equal(heads(a, sl), b)


def test_c5_sample_heads_gaussian_gradient(c5_data):
    """C5 (one GPU, all 1024 heads computed) with dO ~ N(0, 1) (seed 43): the 32 spread
    sample heads (both ends and every 8-way shard's first and last head) against the
    oracle, gradients scaled by max(1, max|ref|); identities on every head."""
    q, k, v, _, _ = c5_data
    do = randn_do(*C5)
    o, lse, dq, dk, dv = gpu_fwd_bwd(q, k, v, do, "fp16")
    idx = [h for h in C5_SAMPLE if h not in set(C5_SHARD)]
    qs, ks, vs, dos = (heads(x, idx) for x in (q, k, v, do))
    eo, el = c_oracle.forward(qs, ks, vs, NT)
    assert maxerr(heads(o, idx), eo) < TOL["fp16"] and maxerr(heads(lse, idx), el) < TOL["fp16"]
    for got, e in zip((dq, dk, dv), c_oracle.backward(qs, ks, vs, eo, dos, el, NT)):
        assert np.isfinite(got).all()
        assert maxerr(heads(got, idx), e) < TOL["fp16"] * max(1.0, float(np.abs(e).max()))
    assert_identities(q, v, do, o, dk, dv)


@pytest.mark.parametrize("chunks", [0, 2, 3])
def test_host_api_shards_on_one_device_small(chunks):
    """Uneven 3-way split (7 heads: 3 + 2 + 2) of a small problem through the host API on
    device 0, against the oracle: the shard offsets of O, LSE (a [heads][S] vector) and
    the gradients; with each shard's H2D / kernels / D2H pipeline over 1 (auto), 2 or 3
    head chunks (HOST_CHUNKS; 3 chunks of a 2-head shard fall back to 2)."""
    B, H, S, D = 1, 7, 300, 64
    q, k, v = fo.cli_inputs(B, H, S, D, seed=5)
    do = np.random.RandomState(6).randn(B, H, S, D).astype(np.float32)
    eo, el = c_oracle.forward(q, k, v, NT)
    edq, edk, edv = c_oracle.backward(q, k, v, eo, do, el, NT)
    fa2amd.tune_set("HOST_SHARDS_ON_DEVICE0", 1)
    fa2amd.tune_set("HOST_CHUNKS", chunks)
    try:
        for precision, tol in (("fp32", 1e-3), ("fp16", 1e-2)):
            o, lse, _ = fa2amd.forward_host(q, k, v, precision, num_devices=3)
            dq, dk, dv, _ = fa2amd.backward_host(q, k, v, o, do, lse, precision, num_devices=3)
            assert maxerr(o, eo) < tol and maxerr(lse, el) < tol
            for got, exp in ((dq, edq), (dk, edk), (dv, edv)):
                assert maxerr(got, exp) < tol * max(1.0, float(np.abs(exp).max())), precision
    finally:
        fa2amd.tune_set(None)


# ---------------------------------------------------------------------------
# Beyond 2^31 elements per tensor: 64-bit offsets everywhere on the path
# ---------------------------------------------------------------------------
def test_tensors_beyond_int32_elements():
    """B1_H4104_S8192_D64: 2.15e9 elements (8.6 GB) per tensor, more than a 32-bit index
    reaches (the reference's own CLI keeps sizes in int, src/main.cpp:27).  fwd + bwd on
    one GPU (inputs drawn on the device, dO = ones); the first, a middle and the last head
    (whose rows start past element 2^31) against the C oracle, every tensor finite."""
    if torch.cuda.get_device_properties(0).total_memory < 100 * 2**30:
        pytest.skip("needs ~70 GB of device memory")
    B, H, S, D = 1, 4104, 8192, 64
    assert B * H * S * D > 2**31
    g = torch.Generator(device="cuda").manual_seed(7)
    q, k, v = (torch.rand(B, H, S, D, device="cuda", generator=g) for _ in range(3))
    ones = torch.ones_like(q)
    o, lse = fa2amd.forward(q, k, v, "fp16")
    dq, dk, dv = fa2amd.backward(q, k, v, o, ones, lse, "fp16")
    torch.cuda.synchronize()
    for name, t in (("o", o), ("lse", lse), ("dq", dq), ("dk", dk), ("dv", dv)):
        assert bool(torch.isfinite(t).all()), name
    idx = [0, H // 2, H - 1]
    sel = lambda t: np.ascontiguousarray(t[0, idx].cpu().numpy())[None]  # noqa: E731
    hq, hk, hv = sel(q), sel(k), sel(v)
    go, gl, gdq, gdk, gdv = sel(o), sel(lse), sel(dq), sel(dk), sel(dv)
    del q, k, v, ones, o, lse, dq, dk, dv
    torch.cuda.empty_cache()
    eo, el = c_oracle.forward(hq, hk, hv, NT)
    h1 = np.ones_like(hq)
    edq, edk, edv = c_oracle.backward(hq, hk, hv, eo, h1, el, NT)
    assert maxerr(go, eo) < TOL["fp16"] and maxerr(gl, el) < TOL["fp16"]
    got = np.concatenate([x.ravel() for x in (gdq, gdk, gdv)])
    assert maxerr(got, np.concatenate([x.ravel() for x in (edq, edk, edv)])) < TOL["fp16"]
    assert_identities(hq, hv, h1, go, gdk, gdv)
