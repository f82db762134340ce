"""Harness-compatible experiment runs and reporting.

Mirrors the reporting side of test_flash_attention2.py (detker/CUDA-Flash-Attention):

* the test configurations (``create_test_configs``, :1365-1405; the sequence-length
  sweep B4_H8_D64, S = 128..4096, :1431-1460);
* one row per (config, kernel) with the harness's metrics (:569-606) and pass rule
  (max-abs < tolerance, no NaN/Inf, :1018-1020), PyTorch CPU / GPU reference rows
  as there (:955-993);
* ``experiment_results.csv`` with the harness's exact columns (:1108-1122) and the
  kernel-comparison plots (:1126-1287; matplotlib only, the reference's seaborn
  styling is not installed here).

Modes (``--mode``, :1466-1469): ``forward``; ``backward`` (the FA2 backward fed
with the PyTorch forward's O and LSE, as the harness does, :898-925); ``both``
(the FA2 forward, then the FA2 backward on the forward's own O and LSE, metrics
summed as in ``_run_test_both``, :608-794).  ``--no-stop-on-failure`` (:1482)
keeps going after a failing row (the default stops, :1091-1095);
``--no-gpu-reference`` (:1488) drops the PyTorch GPU rows.

Kernels: ``fa2`` (the C ABI, precision fp32 / fp16 / bf16), ``fa1``, ``vanilla-attn``
(the comparison baselines, fp32 forward, C ABI) and ``fa2-naive`` (kernels/plain-attn.cu
through its CuPy face, head_dim 64).  Expected values are the
harness's own PyTorch-CPU reference computation (``compute_reference``, :197-208;
backward by autograd with dO = ones, :220-232).

    PYTHONPATH=cuda-flash-attention_amd python -m fa2amd.experiments --mode forward --experiment \
        --save-results --output-dir out/
"""
from __future__ import annotations

import argparse
import csv
import os
import time
from dataclasses import dataclass, field

import numpy as np

CSV_COLUMNS = ["Test", "Kernel", "Type", "Batch", "Heads", "SeqLen", "HeadDim", "Status", "MaxError", "MeanError",
               "MSE", "MaxRelError", "KernelTime_ms", "TorchTime_ms", "Speedup", "TFLOPS", "Bandwidth_GBps",
               "ErrorMessage"]

# test_flash_attention2.py:1371-1399 (name, B, H, S, D)
TEST_CONFIGS = [
    ("Small-1", 1, 1, 128, 64), ("Small-2", 2, 4, 256, 64), ("Small-3", 2, 8, 256, 64),
    ("Medium-1", 2, 8, 512, 64), ("Medium-2", 4, 8, 512, 64),
    ("Large-1", 2, 8, 1024, 64), ("Large-2", 4, 12, 1024, 64),
    ("Edge-NonPowerOf2", 8, 16, 100, 64), ("Edge-SmallSeq", 8, 16, 32, 64),
    ("Stress-1", 8, 16, 2048, 64),
]
SEQLEN_SWEEP = (128, 256, 512, 1024, 2048, 4096)
FORWARD_KERNELS = ("fa2-naive", "vanilla-attn", "fa1", "fa2")  # the harness's experiment set + fa1


@dataclass
class Row:
    test: str
    kernel: str
    type: str
    B: int
    H: int
    S: int
    D: int
    passed: bool = True
    metrics: dict = field(default_factory=dict)
    kernel_ms: float = 0.0
    torch_ms: float = 0.0
    error: str = ""

    def as_csv(self):
        m = self.metrics
        return {"Test": self.test, "Kernel": self.kernel.upper(), "Type": self.type.upper()[:3], "Batch": self.B,
                "Heads": self.H, "SeqLen": self.S, "HeadDim": self.D, "Status": "PASS" if self.passed else "FAIL",
                "MaxError": m.get("max_abs_error", 0.0), "MeanError": m.get("mean_abs_error", 0.0),
                "MSE": m.get("mse", 0.0), "MaxRelError": m.get("max_rel_error", 0.0), "KernelTime_ms": self.kernel_ms,
                "TorchTime_ms": self.torch_ms, "Speedup": m.get("speedup", 0.0), "TFLOPS": m.get("tflops", 0.0),
                "Bandwidth_GBps": m.get("bandwidth_gbps", 0.0), "ErrorMessage": self.error}


def harness_inputs(B, H, S, D, seed=42):
    """The harness's synthetic inputs (generate_test_data(None, cfg), :182-195)."""
    import torch

    g = torch.Generator().manual_seed(seed)
    return tuple(torch.rand(B, H, S, D, generator=g) for _ in range(3))


def torch_reference(q, k, v):
    """compute_reference (:197-208): softmax(Q K^T / sqrt(D)) V on the CPU, and its time."""
    import torch

    t0 = time.perf_counter()
    s = torch.matmul(q, k.transpose(-2, -1)) / (q.shape[-1] ** 0.5)
    o = torch.matmul(torch.softmax(s, dim=-1), v)
    return o, (time.perf_counter() - t0) * 1e3


def torch_reference_backward(q, k, v):
    """compute_reference_backward (:220-232): autograd of sum(O) (dO = ones)."""
    import torch

    qq, kk, vv = (x.clone().requires_grad_() for x in (q, k, v))
    t0 = time.perf_counter()
    o = torch.matmul(torch.softmax(torch.matmul(qq, kk.transpose(-2, -1)) / (q.shape[-1] ** 0.5), dim=-1), vv)
    o.backward(torch.ones_like(o))
    ms = (time.perf_counter() - t0) * 1e3
    return o.detach(), (qq.grad, kk.grad, vv.grad), ms


def _gpu_time(fn, runs=10):
    import torch

    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(runs):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / runs


_BASELINE = None  # hiprtc-compiled baseline modules, built on first use


def run_forward(name, B, H, S, D, kernels, precision="fp32", tolerance=1e-3, gpu_reference=True):
    import torch

    import fa2amd
    from . import harness

    q, k, v = harness_inputs(B, H, S, D)
    exp, torch_ms = torch_reference(q, k, v)
    exp = exp.numpy()
    rows = [Row(name, "pytorch cpu", "forward", B, H, S, D, True,
                {**harness.compute_metrics(exp, exp, torch_ms, torch_ms, B, H, S, D), "speedup": 1.0},
                torch_ms, torch_ms)]
    tq, tk, tv = (x.cuda() for x in (q, k, v))
    if gpu_reference:
        gpu_ms = _gpu_time(lambda: torch.nn.functional.scaled_dot_product_attention(tq, tk, tv))
        og = torch.nn.functional.scaled_dot_product_attention(tq, tk, tv).cpu().numpy()
        rows.append(Row(name, "pytorch gpu", "forward", B, H, S, D, True,
                        harness.compute_metrics(og, exp, gpu_ms, torch_ms, B, H, S, D), gpu_ms, torch_ms))
    for kern in kernels:
        try:
            if kern == "fa2":
                o = torch.empty_like(tq)
                lse = torch.empty((B, H, S), device=tq.device)
                ms = _gpu_time(lambda: fa2amd.forward(tq, tk, tv, precision, out=o, lse=lse))
            elif kern == "fa1":
                o, l, m = fa2amd.fa1_forward(tq, tk, tv)
                ms = _gpu_time(lambda: fa2amd.fa1_forward(tq, tk, tv, out=o, l=l, m=m))
            elif kern == "fa2-naive":
                if D != 64:
                    raise ValueError("fa2-naive is instantiated for head_dim 64 only")
                global _BASELINE
                if _BASELINE is None:
                    _BASELINE = harness.BaselineRawRunner()
                got, ms = _BASELINE.run_naive_fa2_kernel(q, k, v)
                o = torch.from_numpy(got)
            elif kern == "vanilla-attn":
                o, lse, p = fa2amd.naive_forward(tq, tk, tv)
                ms = _gpu_time(lambda: fa2amd.naive_forward(tq, tk, tv, out=o, lse=lse, scores=p))
            else:
                raise ValueError(f"unknown kernel {kern}")
            got = o.cpu().numpy()
            met = harness.compute_metrics(got, exp, ms, torch_ms, B, H, S, D)
            label = kern if (kern != "fa2" or precision == "fp32") else f"fa2-{precision}"
            rows.append(Row(name, label, "forward", B, H, S, D, harness.passed(met, got, tolerance), met, ms,
                            torch_ms))
        except Exception as e:  # recorded as a FAIL row, as the harness does (:1030-1046)
            rows.append(Row(name, kern, "forward", B, H, S, D, False, {}, 0.0, torch_ms, str(e)))
    return rows


def _gpu_reference_grads(q, k, v):
    """PyTorch GPU SDPA forward + autograd backward (dO = ones), one warm-up, one timed
    run (the harness's GPU reference rows, :836-880 and :651-699)."""
    import torch

    def once():
        qq, kk, vv = (x.detach().cuda().requires_grad_() for x in (q, k, v))
        o = torch.nn.functional.scaled_dot_product_attention(qq, kk, vv)
        o.backward(torch.ones_like(o))
        return o, qq.grad, kk.grad, vv.grad

    once()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    o, dq, dk, dv = once()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3
    return o.detach().cpu().numpy(), [g.cpu().numpy() for g in (dq, dk, dv)], ms


def _bwd_metrics(harness, got, exp, ms, torch_ms, B, H, S, D):
    met = harness.compute_metrics(got, exp, ms, torch_ms, B, H, S, D)
    met["tflops"] = 2.5 * 4 * B * H * S * S * D / (ms * 1e-3) / 1e12 if ms > 0 else 0.0  # :634
    return met


def run_backward(name, B, H, S, D, precision="fp32", tolerance=1e-3, gpu_reference=True):
    """--mode backward (:812-940): the FA2 backward is fed the PyTorch forward's O and
    its LSE (natural log, max-shifted, :905-921), as the harness does; dO = ones."""
    import torch

    import fa2amd
    from . import harness

    q, k, v = harness_inputs(B, H, S, D)
    o_ref, grads_ref, torch_ms = torch_reference_backward(q, k, v)
    exp = np.concatenate([g.numpy().ravel() for g in grads_ref])
    cpu_met = _bwd_metrics(harness, exp, exp, torch_ms, torch_ms, B, H, S, D)
    rows = [Row(name, "pytorch cpu", "backward", B, H, S, D, True, {**cpu_met, "speedup": 1.0}, torch_ms, torch_ms)]
    if gpu_reference:
        _, gg, gms = _gpu_reference_grads(q, k, v)
        got = np.concatenate([g.ravel() for g in gg])
        rows.append(Row(name, "pytorch gpu", "backward", B, H, S, D, True,
                        _bwd_metrics(harness, got, exp, gms, torch_ms, B, H, S, D), gms, torch_ms))
    s = torch.matmul(q, k.transpose(-2, -1)) / np.sqrt(D)
    m = s.max(dim=-1, keepdim=True)[0]
    lse = (m.squeeze(-1) + torch.log(torch.exp(s - m).sum(dim=-1))).numpy()
    r = harness.FA2Runner(precision)
    label = "fa2" if precision == "fp32" else f"fa2-{precision}"
    try:
        grads, ms = r.run_cuda_fa2_backward_kernel(q, k, v, o_ref.numpy(), np.ones(q.shape, np.float32), lse)
        got = np.concatenate([grads[n].ravel() for n in ("dQ", "dK", "dV")])
        met = _bwd_metrics(harness, got, exp, ms, torch_ms, B, H, S, D)
        rows.append(Row(name, label, "backward", B, H, S, D, harness.passed(met, got, tolerance), met, ms, torch_ms))
    except Exception as e:  # a FAIL row, as the harness records errors
        rows.append(Row(name, label, "backward", B, H, S, D, False, {}, 0.0, torch_ms, str(e)))
    return rows


def run_both(name, B, H, S, D, precision="fp32", tolerance=1e-3, gpu_reference=True):
    """--mode both (_run_test_both, :608-794): the FA2 forward, then the FA2 backward on
    the forward's own O and LSE.  One row per implementation; the FA2 row passes when
    both the output and the concatenated gradients pass the harness rule, its time is
    forward + backward, TFLOPS counts 3.5x the forward FLOPs (:633-635), bandwidth is
    the sum of the two passes' (:766)."""
    import fa2amd  # noqa: F401  (the C ABI must load)
    from . import harness

    q, k, v = harness_inputs(B, H, S, D)
    o_exp, fwd_ms = torch_reference(q, k, v)
    _, grads_ref, bwd_ms = torch_reference_backward(q, k, v)
    torch_ms = fwd_ms + bwd_ms
    o_exp = o_exp.numpy()
    exp = np.concatenate([g.numpy().ravel() for g in grads_ref])
    total_flops = 3.5 * 4 * B * H * S * S * D
    bytes_ = B * H * S * D * 4 * 4

    def rates(ms):
        return (total_flops / (ms * 1e-3) / 1e12 if ms > 0 else 0.0,
                bytes_ / (ms * 1e-3) / 1e9 if ms > 0 else 0.0)

    tf, bw = rates(torch_ms)
    rows = [Row(name, "pytorch cpu", "both", B, H, S, D, True,
                {"max_abs_error": 0.0, "mean_abs_error": 0.0, "mse": 0.0, "max_rel_error": 0.0, "speedup": 1.0,
                 "tflops": tf, "bandwidth_gbps": bw}, torch_ms, torch_ms)]
    if gpu_reference:
        og, gg, gms = _gpu_reference_grads(q, k, v)
        got = np.concatenate([g.ravel() for g in gg])
        fe, be = np.abs(og - o_exp), np.abs(got - exp)
        tf, bw = rates(gms)
        rows.append(Row(name, "pytorch gpu", "both", B, H, S, D, True,
                        {"max_abs_error": float(max(fe.max(), be.max())),
                         "mean_abs_error": float((fe.mean() + be.mean()) / 2), "mse": 0.0, "max_rel_error": 0.0,
                         "speedup": torch_ms / gms if gms > 0 else 0.0, "tflops": tf, "bandwidth_gbps": bw},
                        gms, torch_ms))
    label = "fa2" if precision == "fp32" else f"fa2-{precision}"
    try:
        r = harness.FA2Runner(precision)
        out, lse, f_ms = r.run_fa2_forward_kernel(q, k, v)
        fm = harness.compute_metrics(out, o_exp, f_ms, fwd_ms, B, H, S, D)
        fwd_ok = harness.passed(fm, out, tolerance)
        grads, b_ms = r.run_cuda_fa2_backward_kernel(q, k, v, out, np.ones(q.shape, np.float32), lse)
        got = np.concatenate([grads[n].ravel() for n in ("dQ", "dK", "dV")])
        bm = harness.compute_metrics(got, exp, b_ms, bwd_ms, B, H, S, D)
        bwd_ok = harness.passed(bm, got, tolerance)
        ms = f_ms + b_ms
        tf, _ = rates(ms)
        met = {"max_abs_error": max(fm["max_abs_error"], bm["max_abs_error"]),
               "mean_abs_error": (fm["mean_abs_error"] + bm["mean_abs_error"]) / 2,
               "mse": (fm["mse"] + bm["mse"]) / 2, "max_rel_error": max(fm["max_rel_error"], bm["max_rel_error"]),
               "speedup": torch_ms / ms if ms > 0 else 0.0, "tflops": tf,
               "bandwidth_gbps": fm["bandwidth_gbps"] + bm["bandwidth_gbps"],
               "fwd_max_abs_error": fm["max_abs_error"], "bwd_max_abs_error": bm["max_abs_error"],
               "fwd_ms": f_ms, "bwd_ms": b_ms}
        err = ""
        if not fwd_ok:
            err += f"Forward failed (err={fm['max_abs_error']:.2e}). "
        if not bwd_ok:
            err += f"Backward failed (err={bm['max_abs_error']:.2e}). "
        rows.append(Row(name, label, "both", B, H, S, D, fwd_ok and bwd_ok, met, ms, torch_ms, err.strip()))
    except Exception as e:
        rows.append(Row(name, label, "both", B, H, S, D, False, {}, 0.0, torch_ms, str(e)))
    return rows


def write_csv(rows, path):
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=CSV_COLUMNS)
        w.writeheader()
        for r in rows:
            w.writerow(r.as_csv())


def plot(rows, out_dir):
    """kernel_comparison.png: time and TFLOPS per test and kernel (the harness's
    _generate_plots panels, :1126-1200).  Skipped if matplotlib is unavailable."""
    try:
        import matplotlib

        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
    except ImportError:
        return None
    ok = [r for r in rows if r.passed and r.kernel_ms > 0]
    tests = list(dict.fromkeys(r.test for r in ok))
    kernels = list(dict.fromkeys(r.kernel for r in ok))
    fig, axes = plt.subplots(1, 2, figsize=(14, 5))
    for kern in kernels:
        xs = [tests.index(r.test) for r in ok if r.kernel == kern]
        axes[0].plot(xs, [r.kernel_ms for r in ok if r.kernel == kern], marker="o", label=kern.upper())
        axes[1].plot(xs, [r.metrics.get("tflops", 0) for r in ok if r.kernel == kern], marker="o",
                     label=kern.upper())
    for ax, title in zip(axes, ("Kernel time (ms)", "TFLOPS")):
        ax.set_xticks(range(len(tests)))
        ax.set_xticklabels(tests, rotation=45, ha="right")
        ax.set_title(title)
        ax.grid(True, alpha=0.3)
        ax.legend()
    axes[0].set_yscale("log")
    fig.tight_layout()
    path = os.path.join(out_dir, "kernel_comparison.png")
    fig.savefig(path, dpi=120)
    plt.close(fig)
    if any("seqlen" in r.test.lower() for r in ok):
        plot_seqlen(ok, out_dir, plt)
    return path


def plot_seqlen(ok, out_dir, plt):
    """seqlen_analysis.png for the SeqLen-* rows: TFLOPS, bandwidth, speedup over
    PyTorch and time against S, one line per kernel (the harness's
    _generate_seqlen_plots, test_flash_attention2.py:1207-1287)."""
    rows = sorted((r for r in ok if "seqlen" in r.test.lower()), key=lambda r: r.S)
    kernels = sorted({r.kernel for r in rows})
    seqs = sorted({r.S for r in rows})
    panels = (("TFLOPS", lambda r: r.metrics.get("tflops", 0.0), "o", False),
              ("Bandwidth (GB/s)", lambda r: r.metrics.get("bandwidth_gbps", 0.0), "s", False),
              ("Speedup vs PyTorch", lambda r: r.metrics.get("speedup", 0.0), "^", False),
              ("Execution Time (ms)", lambda r: r.kernel_ms, "d", True))
    fig, axes = plt.subplots(2, 2, figsize=(16, 12))
    for ax, (label, get, marker, logy) in zip(axes.flat, panels):
        for kern in kernels:
            kr = [r for r in rows if r.kernel == kern]
            ax.plot([r.S for r in kr], [get(r) for r in kr], marker=marker, linewidth=2, markersize=6,
                    label=kern.upper())
        if label.startswith("Speedup"):
            ax.axhline(y=1.0, color="r", linestyle="--", linewidth=1, alpha=0.5)
        ax.set_xlabel("Sequence Length")
        ax.set_ylabel(label)
        ax.set_title(f"{label.split(' (')[0]} vs Sequence Length")
        ax.set_xscale("log", base=2)
        ax.set_xticks(seqs)
        ax.set_xticklabels([str(x) for x in seqs])
        if logy:
            ax.set_yscale("log")
        ax.legend(fontsize=9)
        ax.grid(True, alpha=0.3, which="both")
    fig.suptitle("Sequence Length Scaling Analysis (MI355X)")
    fig.tight_layout()
    path = os.path.join(out_dir, "seqlen_analysis.png")
    fig.savefig(path, dpi=120)
    plt.close(fig)
    return path


CSV_NAME = {"forward": "experiment_results.csv", "backward": "backward_experiment_results.csv",
            "both": "both_experiment_results.csv"}


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--mode", choices=["forward", "backward", "both"], default="forward")
    ap.add_argument("--kernel", choices=["fa2", "fa1", "vanilla-attn", "fa2-naive"], default="fa2")
    ap.add_argument("--precision", choices=["fp32", "fp16", "bf16"], default="fp32")
    ap.add_argument("--experiment", action="store_true", help="every kernel on every test config")
    ap.add_argument("--seqlen-experiment", action="store_true", help="B4_H8_D64, S = 128..4096")
    ap.add_argument("--tolerance", type=float, default=1e-3)
    ap.add_argument("--no-stop-on-failure", action="store_true", help="continue testing after the first failure")
    ap.add_argument("--no-gpu-reference", action="store_true", help="no PyTorch GPU reference rows")
    ap.add_argument("--configs", default="", help="comma-separated subset of config names")
    ap.add_argument("--save-results", action="store_true")
    ap.add_argument("--output-dir", default="./experiment_results")
    args = ap.parse_args(argv)

    # :1494-1495 -- only fa2 has a backward
    if args.mode in ("backward", "both") and args.kernel != "fa2":
        ap.error(f"Only 'fa2' kernel supports backward pass. Got --kernel={args.kernel} with --mode={args.mode}")
    if args.seqlen_experiment:
        configs = [(f"SeqLen-S{s}", 4, 8, s, 64) for s in SEQLEN_SWEEP]
    else:
        configs = TEST_CONFIGS
    if args.configs:
        keep = set(args.configs.split(","))
        configs = [c for c in configs if c[0] in keep]
    forward_set = args.mode == "forward" and (args.experiment or args.seqlen_experiment)
    kernels = FORWARD_KERNELS if forward_set else (args.kernel,)
    gpu_ref = not args.no_gpu_reference
    stop = not args.no_stop_on_failure

    rows = []
    for name, B, H, S, D in configs:
        if args.mode == "forward":
            new = run_forward(name, B, H, S, D, kernels, args.precision, args.tolerance, gpu_ref)
        elif args.mode == "backward":
            new = run_backward(name, B, H, S, D, args.precision, args.tolerance, gpu_ref)
        else:
            new = run_both(name, B, H, S, D, args.precision, args.tolerance, gpu_ref)
        rows += new
        for r in new:
            print(f"{r.test:18s} {r.kernel.upper():14s} {r.type[:3].upper()} {'PASS' if r.passed else 'FAIL'} "
                  f"max_err {r.metrics.get('max_abs_error', float('nan')):.3e} {r.kernel_ms:9.4f} ms "
                  f"{r.metrics.get('tflops', 0.0):8.3f} TFLOPS {r.error}", flush=True)
        if stop and not all(r.passed for r in new):
            print("Stopping on first failure (stop_on_failure=True)", flush=True)  # :1091-1095
            break
    if args.save_results:
        os.makedirs(args.output_dir, exist_ok=True)
        write_csv(rows, os.path.join(args.output_dir, CSV_NAME[args.mode]))
        plot(rows, args.output_dir)
    return 0 if all(r.passed for r in rows) else 1


if __name__ == "__main__":
    raise SystemExit(main())
