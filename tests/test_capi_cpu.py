"""CPU-only checks of the boundary: the C-ABI library loads and exports every
symbol include/fa2_amd.h declares, argument validation needs no GPU, the shard
rule, the CLI's argv/dir contract, and the hiprtc (CuPy-face) compile of the
reference-named kernel files.  No compute call touches a device here."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import fa2amd
from fa2amd import rawmodule

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "fa2_amd.h")


def header_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(fa2_[a-z_0-9]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    L = fa2amd.lib()
    declared = header_functions()
    assert len(declared) >= 10
    for name in declared:
        assert hasattr(L, name), name
    assert sorted(fa2amd.C_SYMBOLS) == declared


def test_version():
    assert fa2amd.version() == 20100


def test_tune_overrides_validated_and_restored():
    """fa2_tune_set rejects names outside the documented knob list (a misspelt knob
    would otherwise leave an A/B on the default plan), and fa2amd.tuned restores the
    overrides that were set before the block, nested blocks included."""
    fa2amd.tune_set(None)
    with pytest.raises(fa2amd.FA2Error, match="unknown knob"):
        fa2amd.tune_set("FWD_WAVE", 4)
    with pytest.raises(fa2amd.FA2Error, match="unknown knob"):
        fa2amd.tune_get("NOPE")
    assert all(fa2amd.tune_get(k) is None for k in fa2amd.KNOBS)
    fa2amd.tune_set("DQ_KS", 2)
    with fa2amd.tuned(DKDV_QS=2, DQ_KS=4):
        assert fa2amd.tune_get("DKDV_QS") == 2 and fa2amd.tune_get("DQ_KS") == 4
        with fa2amd.tuned(FWD_WAVES=4):
            assert fa2amd.tune_get("FWD_WAVES") == 4 and fa2amd.tune_get("DKDV_QS") == 2
        assert fa2amd.tune_get("FWD_WAVES") is None and fa2amd.tune_get("DQ_KS") == 4
    assert fa2amd.tune_get("DQ_KS") == 2 and fa2amd.tune_get("DKDV_QS") is None
    fa2amd.tune_set(None)
    assert fa2amd.tune_get("DQ_KS") is None


def test_invalid_arguments_rejected_without_device():
    L = fa2amd.lib()
    null = ctypes.c_void_p(0)
    one = ctypes.c_void_p(16)
    # bad head_dim
    rc = L.fa2_forward(one, one, one, one, one, 1, 1, 8, 48, fa2amd.FA2_FP16, null)
    assert rc == -1 and b"head_dim" in L.fa2_last_error()
    # bad precision
    rc = L.fa2_forward(one, one, one, one, one, 1, 1, 8, 64, 7, null)
    assert rc == -1 and b"precision" in L.fa2_last_error()
    # null pointer
    rc = L.fa2_backward(one, one, one, one, one, one, one, one, null, one, 1, 1, 8, 64, fa2amd.FA2_FP32, null)
    assert rc == -1 and b"null" in L.fa2_last_error()
    rc = L.fa2_backward_dq_delta(one, one, one, null, one, one, one, one, 1, 1, 8, 64, null)
    assert rc == -1 and b"null" in L.fa2_last_error()
    rc = L.fa2_backward_dq_delta(one, one, one, one, one, one, one, one, 1, 1, 8, 96, null)
    assert rc == -1 and b"head_dim" in L.fa2_last_error()
    # non-positive sizes
    assert L.fa2_delta(one, one, one, 0, 1, 8, 64, null) == -1


@pytest.mark.parametrize("total,shards", [(16, 1), (16, 2), (1024, 8), (7, 3), (3, 8), (64, 4)])
def test_shard_range_c_and_python_agree(total, shards):
    L = fa2amd.lib()
    covered = []
    for i in range(shards):
        f, c = ctypes.c_int(), ctypes.c_int()
        assert L.fa2_shard_range(total, shards, i, ctypes.byref(f), ctypes.byref(c)) == 0
        assert (f.value, c.value) == fa2amd.shard_range(total, shards, i)
        covered.extend(range(f.value, f.value + c.value))
    assert covered == list(range(total))  # contiguous, disjoint, complete


def test_python_api_refuses_cpu_tensors():
    import torch
    q = torch.zeros(1, 1, 8, 64)
    with pytest.raises(fa2amd.FA2Error):
        fa2amd.forward(q, q, q)


@pytest.mark.parametrize("argv,needle", [
    ([], "USAGE"),
    (["fa3", "forward", "fp32", "x/B1_H1_S8_D64"], "USAGE"),
    (["fa2", "both", "fp32", "x/B1_H1_S8_D64"], "USAGE"),
    (["fa2", "forward", "fp8", "x/B1_H1_S8_D64"], "USAGE"),
    (["fa2", "forward", "fp32", "x/not_a_shape"], "sscanf"),
])
def test_cli_argv_contract(argv, needle):
    r = subprocess.run([fa2amd.CLI_PATH] + argv, capture_output=True, text=True, timeout=60)
    assert r.returncode != 0
    assert needle in r.stderr


@pytest.mark.parametrize("fname,symbols", [
    ("kernel_fa2_optimized.cu", ["flash_attention2_forward_kernel_wrapper"]),
    ("f-attn2-backward.cu", ["D_computation_reduction_kernel_wrapper", "flash_attention2_backward_kernel_wrapper"]),
    ("kernel_fa2_optimized_f16.cu", ["flash_attention2_forward_kernel_wrapper"]),
    ("f-attn2-backward_f16.cu", ["D_computation_reduction_kernel_wrapper", "flash_attention2_backward_kernel_wrapper"]),
])
def test_cupy_face_compiles_under_hiprtc(fname, symbols):
    """test_flash_attention2.py:113-145 compiles these files' text with
    ('-std=c++14', '-DCUPY_INLINE_COMPILE'); the same must work here."""
    co = rawmodule.compile_source(rawmodule.load_kernel_source(fname))
    exported = rawmodule.exported_kernels(co)
    for s in symbols:
        assert s in exported


@pytest.mark.parametrize("fname,symbols", [
    ("f-attn.cu", ["flash_attention_forward_kernel_wrapper"]),
    ("vanilla-attn.cu", ["vanilla_attention_kernel_wrapper"]),
    ("plain-attn.cu", ["flash_attention2_forward_kernel_wrapper"]),
])
def test_baseline_cupy_face_compiles_under_hiprtc(fname, symbols):
    """The harness's comparison kernels (test_flash_attention2.py:77-78, 147-170)."""
    co = rawmodule.compile_source(rawmodule.load_kernel_source(fname))
    exported = rawmodule.exported_kernels(co)
    for s in symbols:
        assert s in exported


@pytest.mark.parametrize("argv,needle", [
    (["fa1", "backward", "fp32", "x/B1_H1_S8_D64"], "Flash Attention 1 backward pass not implemented"),
    (["naive", "forward_backward", "fp32", "x/B1_H1_S8_D64"], "Vanilla Attention backward pass not implemented"),
    (["fa1", "forward", "fp16", "x/B1_H1_S8_D64"], "Flash Attention 1 FP16 support not implemented"),
    (["naive", "forward", "fp16", "x/B1_H1_S8_D64"], "Vanilla Attention FP16 support not implemented"),
])
def test_cli_baseline_contract(tmp_path, argv, needle):
    """The reference's messages for the baselines' unsupported combinations
    (include/dispatcher.h:31-50, 74-83), reached before any GPU work (inputs exist)."""
    d = tmp_path / "B1_H1_S8_D64"
    d.mkdir()
    for n in ("Q", "K", "V", "O", "logsumexp"):
        np.zeros(8 * 64 if n != "logsumexp" else 8, np.float32).tofile(d / f"{n}.bin")
    argv = argv[:3] + [str(d)]
    r = subprocess.run([fa2amd.CLI_PATH] + argv, capture_output=True, text=True, timeout=60)
    assert r.returncode != 0
    assert needle in r.stderr


@pytest.mark.parametrize("fname,symbols", [
    ("kernel_fa2_optimized_f16.cu", ["flash_attention2_forward_kernel_wrapper"]),
    ("f-attn2-backward_f16.cu", ["D_computation_reduction_kernel_wrapper", "flash_attention2_backward_kernel_wrapper"]),
])
def test_cupy_face_bf16_compiles_under_hiprtc(fname, symbols):
    """The _f16 files' text with -DFA2_TILE_BF16 added: the same symbols, bf16 MFMA."""
    co = rawmodule.compile_source(rawmodule.load_kernel_source(fname),
                                  tuple(rawmodule.HARNESS_OPTIONS) + ("-DFA2_TILE_BF16",))
    exported = rawmodule.exported_kernels(co)
    for s in symbols:
        assert s in exported
    assert co != rawmodule.compile_source(rawmodule.load_kernel_source(fname))  # a different tile type


@pytest.mark.parametrize("suffix", ["", "_f16"])
@pytest.mark.parametrize("D", [32, 64, 128])
def test_cupy_face_lds_budget(D, suffix):
    """static LDS + the harness's dynamic LDS (test_flash_attention2.py:278-281, 522-527)
    must fit the 160 KiB a workgroup may own, for every supported head_dim."""
    fwd = rawmodule.static_lds_bytes(rawmodule.compile_source(
        rawmodule.load_kernel_source(f"kernel_fa2_optimized{suffix}.cu")))
    bwd = rawmodule.static_lds_bytes(rawmodule.compile_source(
        rawmodule.load_kernel_source(f"f-attn2-backward{suffix}.cu")))
    dyn_fwd = (32 * D * 2 + 32 * D + 32 * 32 + 32 * 3) * 4
    dyn_bwd = (32 * D + 32 * D * 4 + 32 + 32 * 32) * 4
    assert fwd["flash_attention2_forward_kernel_wrapper"] + dyn_fwd <= rawmodule.MAX_LDS_BYTES
    assert bwd["flash_attention2_backward_kernel_wrapper"] + dyn_bwd <= rawmodule.MAX_LDS_BYTES
    assert bwd["D_computation_reduction_kernel_wrapper"] + 64 * 4 <= rawmodule.MAX_LDS_BYTES


def test_experiment_csv_columns(tmp_path):
    """experiment_results.csv carries the harness's exact columns (test_flash_attention2.py:1108-1122;
    the header of the reference's plots/experiment_results.csv)."""
    from fa2amd import experiments

    assert experiments.CSV_COLUMNS == [
        "Test", "Kernel", "Type", "Batch", "Heads", "SeqLen", "HeadDim", "Status", "MaxError", "MeanError", "MSE",
        "MaxRelError", "KernelTime_ms", "TorchTime_ms", "Speedup", "TFLOPS", "Bandwidth_GBps", "ErrorMessage"]
    rows = [experiments.Row("Small-1", "fa2", "forward", 1, 1, 128, 64, True,
                            {"max_abs_error": 1e-7, "tflops": 0.5}, 0.01, 1.0),
            experiments.Row("Small-1", "fa1", "forward", 1, 1, 128, 64, False, {}, 0.0, 1.0, "boom")]
    p = tmp_path / "experiment_results.csv"
    experiments.write_csv(rows, str(p))
    lines = p.read_text().splitlines()
    assert lines[0].split(",") == experiments.CSV_COLUMNS
    assert lines[1].startswith("Small-1,FA2,FOR,1,1,128,64,PASS,")
    assert lines[2].startswith("Small-1,FA1,FOR,1,1,128,64,FAIL,") and lines[2].endswith("boom")


def test_experiment_cli_flags(monkeypatch, tmp_path):
    """The harness's --mode both / --no-stop-on-failure / --no-gpu-reference
    (test_flash_attention2.py:1466-1495) and its stop-on-first-failure loop
    (:1091-1095), with the per-config runners stubbed (no GPU here)."""
    from fa2amd import experiments

    with pytest.raises(SystemExit) as e:
        experiments.main(["--mode", "both", "--kernel", "fa1"])
    assert e.value.code == 2
    with pytest.raises(SystemExit):
        experiments.main(["--mode", "backward", "--kernel", "vanilla-attn"])
    calls = []

    def fake(mode):
        def run(name, B, H, S, D, *a):
            gpu_ref = a[-1]
            calls.append((mode, name, gpu_ref))
            ok = name != "Small-2"
            return [experiments.Row(name, "fa2", mode, B, H, S, D, ok, {"max_abs_error": 0.0 if ok else 1.0},
                                    0.1, 1.0)]
        return run

    monkeypatch.setattr(experiments, "run_both", fake("both"))
    monkeypatch.setattr(experiments, "run_backward", fake("backward"))
    monkeypatch.setattr(experiments, "run_forward", fake("forward"))
    cfg = ["--configs", "Small-1,Small-2,Small-3"]
    assert experiments.main(["--mode", "both"] + cfg) == 1
    assert [c[1] for c in calls] == ["Small-1", "Small-2"]  # stopped at the first failure
    assert all(c[2] is True for c in calls)
    calls.clear()
    assert experiments.main(["--mode", "both", "--no-stop-on-failure", "--no-gpu-reference", "--save-results",
                             "--output-dir", str(tmp_path)] + cfg) == 1
    assert [c[1] for c in calls] == ["Small-1", "Small-2", "Small-3"]
    assert all(c[2] is False for c in calls)
    lines = (tmp_path / "both_experiment_results.csv").read_text().splitlines()
    assert [ln.split(",")[2] for ln in lines[1:]] == ["BOT"] * 3
    calls.clear()
    assert experiments.main(["--mode", "backward", "--configs", "Small-1"]) == 0
    assert calls == [("backward", "Small-1", True)]


def test_experiment_seqlen_plot(monkeypatch, tmp_path):
    """--seqlen-experiment --save-results writes seqlen_analysis.png beside the CSV and
    kernel_comparison.png, as the harness's _generate_seqlen_plots does
    (test_flash_attention2.py:1204-1287); runners stubbed (no GPU here)."""
    pytest.importorskip("matplotlib")
    from fa2amd import experiments

    def run(name, B, H, S, D, kernels, *a):
        return [experiments.Row(name, k, "forward", B, H, S, D, True,
                                {"max_abs_error": 0.0, "tflops": 1e-3 * S, "bandwidth_gbps": 1.0, "speedup": 2.0},
                                1e-4 * S, 1.0) for k in kernels]

    monkeypatch.setattr(experiments, "run_forward", run)
    assert experiments.main(["--seqlen-experiment", "--save-results", "--output-dir", str(tmp_path)]) == 0
    for f in ("experiment_results.csv", "kernel_comparison.png", "seqlen_analysis.png"):
        assert (tmp_path / f).stat().st_size > 0, f
    lines = (tmp_path / "experiment_results.csv").read_text().splitlines()
    assert sorted({int(ln.split(",")[5]) for ln in lines[1:]}) == list(experiments.SEQLEN_SWEEP)


def test_bench_traffic_only_from_a_profile_of_the_loaded_build(tmp_path):
    """roofline.traffic comes from profiles/pmc_summary.json only when its _meta.build_id
    is the loaded library's fa2_build_id (a rebuilt kernel cannot inherit old figures)."""
    import json
    import sys

    sys.path.insert(0, ROOT)
    import bench

    bid = fa2amd.build_id()
    assert len(bid) == 16 and bid != "unknown"
    summ = {"_meta": {"S": 2048, "D": 64, "heads": 64, "build_id": bid},
            "fa2_bwd_dkdv_f16_kernel<64,8,1,true,1>": {"hbm_bytes_per_launch": 123.0}}
    p = tmp_path / "pmc.json"
    p.write_text(json.dumps(summ))
    assert bench.traffic_from_profile("dkdv", 64, 2048, 64, bid, str(p)) == 123.0
    assert bench.traffic_from_profile("dkdv", 64, 2048, 64, "0" * 16, str(p)) is None
    assert bench.traffic_from_profile("dkdv", 64, 4096, 64, bid, str(p)) is None
    # the hand-scheduled kernels' entries count too (their names carry <D>)
    summ2 = {"_meta": summ["_meta"], "fa2_bwd_dkdv_hs_kernel<64>": {"hbm_bytes_per_launch": 77.0},
             "fa2_fwd_hs_kernel<64>": {"hbm_bytes_per_launch": 55.0}}
    p.write_text(json.dumps(summ2))
    assert bench.traffic_from_profile("dkdv", 64, 2048, 64, bid, str(p)) == 77.0
    assert bench.traffic_from_profile("fwd", 64, 2048, 64, bid, str(p)) == 55.0
    summ["_meta"].pop("build_id")
    p.write_text(json.dumps(summ))
    assert bench.traffic_from_profile("dkdv", 64, 2048, 64, bid, str(p)) is None


def test_no_float_atomics_on_any_fa2_path():
    """dQ is written once on every face and precision (the reference adds it with
    atomicAdd, f-attn2-backward.cu:298 / f-attn2-backward_f16.cu:289): no kernel source
    of the library issues a float atomic, so every output is bitwise repeatable."""
    kdir = os.path.join(os.path.dirname(fa2amd.LIB_PATH), "..", "kernels")
    pat = re.compile(r"\batomicAdd\s*\(|__hip_atomic_fetch_add|unsafeAtomicAdd|global_atomic_add")
    for name in sorted(os.listdir(kdir)):
        if name.endswith((".cu", ".cuh", ".inc")):
            with open(os.path.join(kdir, name)) as f:
                assert not pat.search(f.read()), name
