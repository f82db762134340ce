"""GPU parity of the comparison baselines: the naive attention of
kernels/vanilla-attn.cu and the FlashAttention-1 forward of kernels/f-attn.cu,
against the oracle, through the C ABI, the CLI (methods ``naive`` / ``fa1``) and
the harness's CuPy launch geometry.  Both are exact-fp32 paths: the reference's
1e-3 harness tolerance (test_flash_attention2.py:1018-1020) and a 2e-5 regression
bound, as for the fp32 FA2 path.
"""
import os
import subprocess

import numpy as np
import pytest

torch = pytest.importorskip("torch")

import fa2amd  # noqa: E402
from fa2amd import harness  # noqa: E402
from oracle import fa2_oracle as fo  # noqa: E402

pytestmark = pytest.mark.gpu

TIGHT = 2e-5
SHAPES = [(1, 2, 100, 64), (2, 2, 64, 32), (1, 2, 77, 128), (2, 4, 256, 64), (1, 1, 33, 32)]


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    fa2amd.lib()


def maxerr(a, b):
    return float(np.abs(np.asarray(a, np.float64) - np.asarray(b, np.float64)).max())


def softmax_rows(q, k):
    s = np.einsum("bhqd,bhkd->bhqk", q.astype(np.float64), k.astype(np.float64)) / np.sqrt(q.shape[-1])
    s -= s.max(-1, keepdims=True)
    p = np.exp(s)
    return p / p.sum(-1, keepdims=True)


@pytest.mark.parametrize("shape", SHAPES)
def test_naive_forward(shape):
    q, k, v = fo.harness_inputs(*shape)
    eo, el = fo.attention_forward(q, k, v)
    o, lse, p = fa2amd.naive_forward(*(torch.from_numpy(x).cuda() for x in (q, k, v)))
    torch.cuda.synchronize()
    assert maxerr(o.cpu().numpy(), eo) < TIGHT
    assert maxerr(lse.cpu().numpy(), el) < TIGHT * 10
    assert maxerr(p.cpu().numpy(), softmax_rows(q, k)) < TIGHT  # the materialised P


@pytest.mark.parametrize("shape", SHAPES)
def test_fa1_forward(shape):
    q, k, v = fo.cli_inputs(*shape, seed=11)
    eo, el = fo.attention_forward(q, k, v)
    o, l, m = fa2amd.fa1_forward(*(torch.from_numpy(x).cuda() for x in (q, k, v)))
    torch.cuda.synchronize()
    assert maxerr(o.cpu().numpy(), eo) < TIGHT
    # the FA1 outputs are (l, m) with LSE = m + ln l (f-attn.cu:167, :200 of the reference)
    lse = m.cpu().numpy().astype(np.float64) + np.log(l.cpu().numpy().astype(np.float64))
    assert maxerr(lse, el) < TIGHT * 10
    s = np.einsum("bhqd,bhkd->bhqk", q.astype(np.float64), k.astype(np.float64)) / np.sqrt(q.shape[-1])
    assert maxerr(m.cpu().numpy(), s.max(-1)) < TIGHT * 10  # m is the row max


def test_baselines_agree_with_fa2_at_c1():
    """C1 = B2_H8_S512_D64 (harness inputs): FA2 fp32, FA1 and naive give the same O."""
    q, k, v = fo.harness_inputs(2, 8, 512, 64)
    tq, tk, tv = (torch.from_numpy(x).cuda() for x in (q, k, v))
    o2, _ = fa2amd.forward(tq, tk, tv, "fp32")
    o1, _, _ = fa2amd.fa1_forward(tq, tk, tv)
    on, _, _ = fa2amd.naive_forward(tq, tk, tv)
    torch.cuda.synchronize()
    eo, _ = fo.attention_forward(q, k, v)
    for o in (o2, o1, on):
        assert maxerr(o.cpu().numpy(), eo) < TIGHT


@pytest.fixture(scope="module")
def baseline_runner():
    return harness.BaselineRawRunner()


@pytest.mark.parametrize("shape", [(1, 2, 128, 64), (2, 2, 100, 64), (1, 4, 512, 64)])
def test_cupy_face_fa1_and_naive(baseline_runner, shape):
    """The harness's run_cuda_fa1_kernel / run_cuda_naive_kernel launches (grid B*H,
    256 / 128 threads, zero-filled outputs) and its pass rule."""
    B, H, S, D = shape
    q, k, v = fo.harness_inputs(B, H, S, D)
    eo, el = fo.attention_forward(q, k, v)
    Q, K, V = (torch.from_numpy(x) for x in (q, k, v))
    out, ms = baseline_runner.run_cuda_fa1_kernel(Q, K, V)
    assert ms > 0 and harness.passed(harness.compute_metrics(out, eo, ms, 1.0, B, H, S, D), out, 1e-3)
    assert maxerr(out, eo) < TIGHT
    lse = baseline_runner.last_m.astype(np.float64) + np.log(baseline_runner.last_l.astype(np.float64))
    assert maxerr(lse, el) < TIGHT * 10
    out, ms = baseline_runner.run_naive_fa2_kernel(Q, K, V)
    assert ms > 0 and harness.passed(harness.compute_metrics(out, eo, ms, 1.0, B, H, S, D), out, 1e-3)
    assert maxerr(out, eo) < 1e-5 and maxerr(baseline_runner.last_lse, el) < 1e-4
    out, ms = baseline_runner.run_cuda_naive_kernel(Q, K, V)
    assert ms > 0 and harness.passed(harness.compute_metrics(out, eo, ms, 1.0, B, H, S, D), out, 1e-3)
    assert maxerr(out, eo) < TIGHT
    assert maxerr(baseline_runner.last_p, softmax_rows(q, k)) < TIGHT


@pytest.mark.parametrize("method", ["naive", "fa1"])
def test_cli_baseline_forward(tmp_path, method):
    """FlashAttention <naive|fa1> forward fp32 <dir>: O.bin as the reference CLI writes it."""
    B, H, S, D = 1, 2, 64, 32
    q, k, v = fo.cli_inputs(B, H, S, D)
    run = tmp_path / f"B{B}_H{H}_S{S}_D{D}"
    run.mkdir()
    for n, x in (("Q", q), ("K", k), ("V", v)):
        x.tofile(run / f"{n}.bin")
    r = subprocess.run([fa2amd.CLI_PATH, method, "forward", "fp32", str(run)], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    eo, el = fo.attention_forward(q, k, v)
    assert maxerr(np.fromfile(run / "O.bin", dtype=np.float32).reshape(q.shape), eo) < TIGHT
    lse_file = np.fromfile(run / "logsumexp.bin", dtype=np.float32).reshape(q.shape[:3])
    if method == "naive":
        assert maxerr(lse_file, el) < TIGHT * 10
    else:  # FA1's `logsumexp` output is the row sum l (>= 1: the max term contributes 1)
        assert (lse_file >= 1.0 - 1e-6).all()


def test_experiment_run_writes_harness_csv(tmp_path):
    """python -m fa2amd.experiments --experiment --save-results on two small configs:
    every kernel row PASSes the harness rule and the CSV / plot are written."""
    from fa2amd import experiments

    rc = experiments.main(["--mode", "forward", "--experiment", "--configs", "Small-1,Edge-NonPowerOf2",
                           "--save-results", "--output-dir", str(tmp_path)])
    assert rc == 0
    text = (tmp_path / "experiment_results.csv").read_text().splitlines()
    assert text[0].split(",") == experiments.CSV_COLUMNS
    kernels = {line.split(",")[1] for line in text[1:]}
    assert {"FA2", "FA1", "VANILLA-ATTN", "FA2-NAIVE", "PYTORCH CPU", "PYTORCH GPU"} <= kernels
    assert all(",PASS," in line for line in text[1:])
    rc = experiments.main(["--mode", "backward", "--configs", "Small-2", "--precision", "fp16", "--tolerance", "1e-2",
                           "--save-results", "--output-dir", str(tmp_path)])
    assert rc == 0
    assert (tmp_path / "backward_experiment_results.csv").exists()


@pytest.mark.parametrize("precision,tol", [("fp32", 1e-3), ("fp16", 1e-2)])
def test_experiment_mode_both(tmp_path, precision, tol):
    """--mode both (_run_test_both, test_flash_attention2.py:608-794): the FA2 forward,
    then the FA2 backward on its own O and LSE; the FA2 row passes the harness rule on
    the output AND the concatenated gradients; CPU and GPU reference rows beside it."""
    from fa2amd import experiments

    rows = experiments.run_both("Edge-NonPowerOf2", 2, 4, 100, 64, precision, tol)
    kinds = [r.kernel for r in rows]
    assert kinds[:2] == ["pytorch cpu", "pytorch gpu"] and kinds[2].startswith("fa2")
    fa2 = rows[2]
    assert fa2.passed, fa2.error
    assert fa2.metrics["fwd_max_abs_error"] < tol and fa2.metrics["bwd_max_abs_error"] < tol
    assert fa2.kernel_ms == pytest.approx(fa2.metrics["fwd_ms"] + fa2.metrics["bwd_ms"])
    rc = experiments.main(["--mode", "both", "--configs", "Small-1,Edge-SmallSeq", "--precision", precision,
                           "--tolerance", str(tol), "--no-gpu-reference", "--save-results", "--output-dir",
                           str(tmp_path)])
    assert rc == 0
    lines = (tmp_path / "both_experiment_results.csv").read_text().splitlines()[1:]
    assert len(lines) == 4 and all(",BOT," in ln and ",PASS," in ln for ln in lines)
    assert not any("PYTORCH GPU" in ln for ln in lines)


def test_experiment_mode_backward_uses_torch_forward():
    """--mode backward feeds the FA2 backward the PyTorch forward's O and LSE (:898-925)."""
    from fa2amd import experiments

    rows = experiments.run_backward("Small-2", 2, 4, 256, 64, "fp32", 1e-3, gpu_reference=False)
    assert [r.kernel for r in rows] == ["pytorch cpu", "fa2"]
    assert rows[1].passed, rows[1].error
