"""Pin the CPU oracle (oracle/) against golden vectors produced by the reference
harness itself (tests/golden/make_golden.py).  CPU only."""
import json
import hashlib
import os

import numpy as np
import pytest

from oracle import fa2_oracle as fo
from oracle import c_oracle as co

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
with open(os.path.join(GOLDEN, "manifest.json")) as _f:
    MANIFEST = json.load(_f)
CASES = sorted(MANIFEST["cases"])


def load(name):
    return dict(np.load(os.path.join(GOLDEN, name + ".npz")))


@pytest.mark.parametrize("name", CASES)
def test_generators_reproduce_reference_inputs(name):
    g, meta = load(name), MANIFEST["cases"][name]
    gen = fo.harness_inputs if meta["dist"] == "harness" else fo.cli_inputs
    q, k, v = gen(meta["B"], meta["H"], meta["S"], meta["D"], seed=meta["seed"])
    np.testing.assert_array_equal(q, g["q"])
    np.testing.assert_array_equal(k, g["k"])
    np.testing.assert_array_equal(v, g["v"])


@pytest.mark.parametrize("name", CASES)
def test_numpy_oracle_forward(name):
    g = load(name)
    o, lse = fo.attention_forward(g["q"], g["k"], g["v"])
    np.testing.assert_allclose(o, g["o"], atol=2e-6, rtol=0)
    np.testing.assert_allclose(lse, g["lse"], atol=2e-5, rtol=0)


@pytest.mark.parametrize("name", CASES)
@pytest.mark.parametrize("grad", ["ones", "rand"])
def test_numpy_oracle_backward(name, grad):
    g = load(name)
    do = np.ones_like(g["q"]) if grad == "ones" else g["do_rand"]
    dq, dk, dv, dl = fo.attention_backward(g["q"], g["k"], g["v"], do)
    scale = max(1.0, float(np.abs(g["dv_" + grad]).max()))
    for ours, key in ((dq, "dq_"), (dk, "dk_"), (dv, "dv_")):
        np.testing.assert_allclose(ours, g[key + grad], atol=2e-6 * scale, rtol=0)
    np.testing.assert_allclose(dl, g["delta_" + grad], atol=1e-4, rtol=1e-5)


@pytest.mark.parametrize("name", CASES)
def test_c_oracle_matches_golden(name):
    g = load(name)
    o, lse = co.forward(g["q"], g["k"], g["v"], nthreads=4)
    np.testing.assert_allclose(o, g["o"], atol=2e-6, rtol=0)
    np.testing.assert_allclose(lse, g["lse"], atol=2e-5, rtol=0)
    dq, dk, dv = co.backward(g["q"], g["k"], g["v"], g["o"], g["do_rand"], g["lse"], nthreads=4)
    scale = max(1.0, float(np.abs(g["dv_rand"]).max()))
    np.testing.assert_allclose(dq, g["dq_rand"], atol=1e-5 * scale, rtol=0)
    np.testing.assert_allclose(dk, g["dk_rand"], atol=1e-5 * scale, rtol=0)
    np.testing.assert_allclose(dv, g["dv_rand"], atol=1e-5 * scale, rtol=0)
    np.testing.assert_allclose(co.delta(g["do_rand"], g["o"]), g["delta_rand"], atol=1e-4, rtol=1e-5)


@pytest.mark.parametrize("name", ["harness_B2_H2_S100_D64", "cli_B1_H2_S64_D64"])
def test_tile_emulator(name):
    """The tile-faithful emulator (fp32 storage) equals the math oracle; with the
    _f16 kernel's rounding points it stays inside the north-star 1e-2 budget."""
    g = load(name)
    o, lse = fo.attention_forward_tiled(g["q"], g["k"], g["v"])
    np.testing.assert_allclose(o, g["o"], atol=1e-5, rtol=0)
    np.testing.assert_allclose(lse, g["lse"], atol=1e-5, rtol=0)
    o16, lse16 = fo.attention_forward_tiled(g["q"], g["k"], g["v"], storage=np.float16)
    assert np.abs(o16 - g["o"]).max() < 1e-2


def test_c1_input_digests_match_reference():
    ent = MANIFEST["digests"]["C1_B2_H8_S512_D64"]
    q, k, v = fo.harness_inputs(2, 8, 512, 64)
    for t, name in ((q, "q"), (k, "k"), (v, "v")):
        assert hashlib.sha256(t.tobytes()).hexdigest() == ent["sha256_" + name]
    o, lse = fo.attention_forward(q, k, v)
    assert abs(float(o.astype(np.float64).sum()) - ent["o_sum"]) < 1e-3 * abs(ent["o_sum"]) * 1e-3
    assert abs(float(lse.astype(np.float64).sum()) - ent["lse_sum"]) < 1e-2


def test_flop_and_byte_accounting():
    # C3 = B4_H16_S2048_D64 -> 68.72 GF fwd, 240.5 GF f+b, 134.2 MB fwd bytes
    assert abs(fo.fwd_flops(4, 16, 2048, 64) / 1e9 - 68.72) < 0.01
    assert abs((fo.fwd_flops(4, 16, 2048, 64) + fo.bwd_flops(4, 16, 2048, 64)) / 1e9 - 240.5) < 0.1
    assert abs(fo.fwd_bytes(4, 16, 2048, 64) / 1e6 - 134.7) < 0.6
