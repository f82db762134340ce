"""Host code under AddressSanitizer (SURVEY §5 "Race detection / sanitizers"; no GPU).

`make asan` builds, with `-fsanitize=address` on the host side only:
* tests/native/capi_check.cpp linked with csrc/capi.cpp -- the C ABI's argument
  validation, shard rule, thread-local errors, the launch-plan table under
  concurrent writers and the host API's no-device error path (leak checking on);
* the CLI (src/main.cpp, src/utils.cpp) -- argv, directory-name and .bin-file
  handling, including missing and short files, and the forward_backward path up to
  the device call;
* tests/native/oracle_check.c linked with oracle/fa2_oracle.c -- the threaded C
  restatement of the oracle on ragged shapes.
A memory error makes ASan abort the binary with a report on stderr.
"""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "cuda-flash-attention_amd")
ASAN_BIN = os.path.join(PKG, "build", "asan")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:exitcode=99")


@pytest.fixture(scope="module")
def built():
    subprocess.run(["make", "-s", "-j8", "-C", PKG, "asan"], check=True, capture_output=True)
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan"], check=True, capture_output=True)


def run(cmd, **kw):
    p = subprocess.run(cmd, env=ENV, capture_output=True, text=True, timeout=300, **kw)
    assert "AddressSanitizer" not in p.stderr, p.stderr[-4000:]
    assert "LeakSanitizer" not in p.stderr, p.stderr[-4000:]
    return p


def test_capi_host_code(built):
    p = run([os.path.join(ASAN_BIN, "capi_check")])
    assert p.returncode == 0, p.stdout + p.stderr
    assert "capi_check: ok" in p.stdout


def test_oracle_c(built):
    p = run([os.path.join(ROOT, "oracle", "build", "asan", "oracle_check")])
    assert p.returncode == 0, p.stdout + p.stderr
    assert "oracle_check: ok" in p.stdout


def _write(d, names, n):
    rng = np.random.default_rng(0)
    for f in names:
        rng.random(n, dtype=np.float32).tofile(os.path.join(d, f + ".bin"))


def test_cli_paths(built, tmp_path):
    cli = os.path.join(ASAN_BIN, "FlashAttention")
    p = run([cli])
    assert p.returncode == 1 and "USAGE" in p.stdout + p.stderr
    p = run([cli, "fa2", "sideways", "fp16", str(tmp_path / "B1_H1_S8_D64")])
    assert p.returncode == 1 and "USAGE" in p.stdout + p.stderr
    p = run([cli, "fa2", "forward", "fp16", str(tmp_path / "not_a_shape")])
    assert p.returncode == 1 and "sscanf" in p.stderr
    d = tmp_path / "B1_H2_S33_D64"
    d.mkdir()
    p = run([cli, "fa2", "forward", "fp16", str(d)])
    assert p.returncode == 1 and "Data files not found" in p.stdout + p.stderr
    n = 2 * 33 * 64
    _write(d, "QV", n)
    np.zeros(n - 5, np.float32).tofile(d / "K.bin")  # short file
    p = run([cli, "fa2", "forward", "fp16", str(d) + "/"])
    assert p.returncode == 1 and "fread" in p.stderr
    _write(d, "K", n)
    # backward needs O.bin and logsumexp.bin
    p = run([cli, "fa2", "backward", "fp32", str(d)])
    assert p.returncode == 1 and "Data files not found" in p.stdout + p.stderr
    _write(d, ["O", "logsumexp"], n)
    np.zeros(2 * 33 - 1, np.float32).tofile(d / "logsumexp.bin")  # short LSE
    p = run([cli, "fa2", "backward", "fp32", str(d)])
    assert p.returncode == 1 and "fread" in p.stderr
    # a complete input set loads; without a GPU the run then stops at the device
    _write(d, ["logsumexp"], 2 * 33)
    p = run([cli, "fa2", "forward_backward", "fp16", str(d)])
    assert "Data loaded successfully" in p.stdout
    if p.returncode != 0:
        assert "HIP error" in p.stderr or "hip" in p.stderr.lower()
    p = run([cli, "naive", "backward", "fp32", str(d)])
    assert p.returncode == 1 and "not implemented" in p.stdout + p.stderr
