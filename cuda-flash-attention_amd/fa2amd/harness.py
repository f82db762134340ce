"""Runners with the reference harness's method names, argument meaning and timing.

Mirrors ``FlashAttention2Tester`` of test_flash_attention2.py (detker/CUDA-Flash-
Attention) for the FA2 path:

* ``run_fa2_forward_kernel(Q, K, V)`` -> ``(output_np, logsumexp_np, elapsed_ms)``
  (test_flash_attention2.py:252-313): CPU torch tensors in, H2D, one warm-up
  launch, mean of 10 timed launches between events, D2H.
* ``run_cuda_fa2_backward_kernel(Q, K, V, output, grad_output, logsumexp)`` ->
  ``({'dQ','dK','dV'}, elapsed_ms)`` (:476-567): Δ computed once untimed, one
  warm-up, then 10 x [zero dQ/dK/dV + backward] timed.
* ``compute_metrics`` (:569-606) with the harness's formulas.

Two back ends:
* ``FA2Runner``     -- the C ABI (libfa2amd.so), precision "fp32" or "fp16";
* ``RawModuleRunner`` -- the reference-named kernel files compiled from source
  text with hiprtc and launched with the harness's exact geometry (CuPy face).

and, for the harness's comparison kernels (``--kernel fa1|vanilla-attn``),
``BaselineRawRunner.run_cuda_fa1_kernel`` / ``run_naive_fa2_kernel`` /
``run_cuda_naive_kernel`` (:315-372, :374-426, :428-474) over kernels/f-attn.cu,
kernels/plain-attn.cu and kernels/vanilla-attn.cu.
"""
from __future__ import annotations

import numpy as np

from . import backward as _backward, delta as _delta, forward as _forward

NUM_RUNS = 10


def _to_dev(t):
    import torch

    return torch.as_tensor(np.ascontiguousarray(t.detach().numpy() if isinstance(t, torch.Tensor) else t)).cuda()


class FA2Runner:
    def __init__(self, precision: str = "fp32"):
        self.precision = precision

    def run_fa2_forward_kernel(self, Q, K, V):
        import torch

        q, k, v = _to_dev(Q), _to_dev(K), _to_dev(V)
        o = torch.zeros_like(q)
        lse = torch.zeros(q.shape[:3], device=q.device, dtype=torch.float32)
        _forward(q, k, v, self.precision, out=o, lse=lse)
        torch.cuda.synchronize()
        start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        start.record()
        for _ in range(NUM_RUNS):
            _forward(q, k, v, self.precision, out=o, lse=lse)
        end.record()
        end.synchronize()
        return o.cpu().numpy(), lse.cpu().numpy(), start.elapsed_time(end) / NUM_RUNS

    def run_cuda_fa2_backward_kernel(self, Q, K, V, output, grad_output, logsumexp):
        import torch

        q, k, v, o, do, lse = (_to_dev(x) for x in (Q, K, V, output, grad_output, logsumexp))
        dq, dk, dv = torch.zeros_like(q), torch.zeros_like(q), torch.zeros_like(q)
        dl = torch.zeros(q.shape[:3], device=q.device, dtype=torch.float32)
        _backward(q, k, v, o, do, lse, self.precision, dq=dq, dk=dk, dv=dv, delta_buf=dl)
        torch.cuda.synchronize()
        start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        start.record()
        for _ in range(NUM_RUNS):
            dq.zero_(); dk.zero_(); dv.zero_()
            _backward(q, k, v, o, do, lse, self.precision, dq=dq, dk=dk, dv=dv, delta_buf=dl)
        end.record()
        end.synchronize()
        grads = {"dQ": dq.cpu().numpy(), "dK": dk.cpu().numpy(), "dV": dv.cpu().numpy()}
        return grads, start.elapsed_time(end) / NUM_RUNS


class RawModuleRunner:
    """Drives kernels/kernel_fa2_optimized.cu and kernels/f-attn2-backward.cu exactly
    as test_flash_attention2.py does through cp.RawModule (the harness names the fp32
    files only, :75-76; the _f16 files export the same symbols and can be passed).
    ``extra_options`` are appended to the harness's hiprtc options: the _f16 files
    compiled with ``-DFA2_TILE_BF16`` run bf16 tiles behind the same symbols."""

    BLOCK_SIZE_R = 32
    BLOCK_SIZE_C = 32

    def __init__(self, fwd_file="kernel_fa2_optimized.cu", bwd_file="f-attn2-backward.cu", extra_options=()):
        from .rawmodule import HARNESS_OPTIONS, RawModule, load_kernel_source

        opts = tuple(HARNESS_OPTIONS) + tuple(extra_options)
        self.fwd_mod = RawModule(load_kernel_source(fwd_file), options=opts,
                                 name_expressions=("flash_attention2_forward_kernel_wrapper",))
        self.bwd_mod = RawModule(load_kernel_source(bwd_file), options=opts, name_expressions=(
            "flash_attention2_backward_kernel_wrapper", "D_computation_reduction_kernel_wrapper"))
        self.fa2_kernel = self.fwd_mod.get_function("flash_attention2_forward_kernel_wrapper")
        self.backward_kernel = self.bwd_mod.get_function("flash_attention2_backward_kernel_wrapper")
        self.d_kernel = self.bwd_mod.get_function("D_computation_reduction_kernel_wrapper")

    def run_fa2_forward_kernel(self, Q, K, V):
        import torch

        B, H, S, D = Q.shape
        q, k, v = _to_dev(Q), _to_dev(K), _to_dev(V)
        o = torch.zeros_like(q)
        lse = torch.zeros((B, H, S), device=q.device, dtype=torch.float32)
        T_r = (S + self.BLOCK_SIZE_R - 1) // self.BLOCK_SIZE_R
        shared_mem = (self.BLOCK_SIZE_R * D * 2 + self.BLOCK_SIZE_C * D + self.BLOCK_SIZE_R * self.BLOCK_SIZE_C
                      + self.BLOCK_SIZE_R * 3) * 4  # = 29056 at D=64 (test_flash_attention2.py:278-281)
        args = (q, k, v, o, lse, B, H, S, D)
        self.fa2_kernel((B * H * T_r,), (256,), args, shared_mem=shared_mem)
        torch.cuda.synchronize()
        start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        start.record()
        for _ in range(NUM_RUNS):
            self.fa2_kernel((B * H * T_r,), (256,), args, shared_mem=shared_mem)
        end.record()
        end.synchronize()
        return o.cpu().numpy(), lse.cpu().numpy(), start.elapsed_time(end) / NUM_RUNS

    def run_cuda_fa2_backward_kernel(self, Q, K, V, output, grad_output, logsumexp):
        import torch

        B, H, S, D = Q.shape
        q, k, v, o, do, lse = (_to_dev(x) for x in (Q, K, V, output, grad_output, logsumexp))
        dq, dk, dv = torch.zeros_like(q), torch.zeros_like(q), torch.zeros_like(q)
        d = torch.zeros((B, H, S), device=q.device, dtype=torch.float32)
        self.d_kernel((B * H * S,), (64,), (do, o, B, H, S, D, d), shared_mem=64 * 4)
        torch.cuda.synchronize()
        T_c = (S + self.BLOCK_SIZE_C - 1) // self.BLOCK_SIZE_C
        shared_mem = (self.BLOCK_SIZE_R * D + self.BLOCK_SIZE_C * D * 4 + self.BLOCK_SIZE_R
                      + self.BLOCK_SIZE_R * self.BLOCK_SIZE_C) * 4  # = 45184 at D=64 (:522-527)
        args = (q, k, v, o, do, lse, d, dq, dk, dv, B, H, S, D)
        self.backward_kernel((B * H * T_c,), (256,), args, shared_mem=shared_mem)
        torch.cuda.synchronize()
        start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        start.record()
        for _ in range(NUM_RUNS):
            dq.zero_(); dk.zero_(); dv.zero_()
            self.backward_kernel((B * H * T_c,), (256,), args, shared_mem=shared_mem)
        end.record()
        end.synchronize()
        grads = {"dQ": dq.cpu().numpy(), "dK": dk.cpu().numpy(), "dV": dv.cpu().numpy()}
        return grads, start.elapsed_time(end) / NUM_RUNS


class BaselineRawRunner:
    """The harness's FA1 and naive-attention runs (test_flash_attention2.py:315-372,
    :428-474): kernels/f-attn.cu and kernels/vanilla-attn.cu compiled from text,
    grid B*H, 256 / 128 threads, zero-filled outputs, head_dim 64 (the wrappers'
    fixed D, as in the reference).  Each returns ``(output_np, elapsed_ms)``."""

    def __init__(self):
        from .rawmodule import RawModule, load_kernel_source

        self.fa1_mod = RawModule(load_kernel_source("f-attn.cu"),
                                 name_expressions=("flash_attention_forward_kernel_wrapper",))
        self.naive_mod = RawModule(load_kernel_source("vanilla-attn.cu"),
                                   name_expressions=("vanilla_attention_kernel_wrapper",))
        self.plain_mod = RawModule(load_kernel_source("plain-attn.cu"),
                                   name_expressions=("flash_attention2_forward_kernel_wrapper",))
        self.fa1_kernel = self.fa1_mod.get_function("flash_attention_forward_kernel_wrapper")
        self.naive_kernel = self.naive_mod.get_function("vanilla_attention_kernel_wrapper")
        self.forward_fa_naive = self.plain_mod.get_function("flash_attention2_forward_kernel_wrapper")

    @staticmethod
    def _timed(fn):
        import torch

        fn()
        torch.cuda.synchronize()
        start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        start.record()
        for _ in range(NUM_RUNS):
            fn()
        end.record()
        end.synchronize()
        return start.elapsed_time(end) / NUM_RUNS

    def run_cuda_fa1_kernel(self, Q, K, V):
        import torch

        B, H, S, D = Q.shape
        if D != 64:
            raise ValueError("the FA1 wrapper is instantiated for head_dim 64 (f-attn.cu:295 in the reference)")
        q, k, v = _to_dev(Q), _to_dev(K), _to_dev(V)
        o = torch.zeros_like(q)
        lse = torch.zeros((B, H, S), device=q.device, dtype=torch.float32)
        maxes = torch.zeros((B, H, S), device=q.device, dtype=torch.float32)
        shared_mem = (32 * D * 2 + 32 * D * 2 + 32 * 32 + 32 * 2) * 4  # :338-341
        ms = self._timed(lambda: self.fa1_kernel((B * H,), (256,), (q, k, v, o, lse, maxes, B, H, S),
                                                 shared_mem=shared_mem))
        self.last_l, self.last_m = lse.cpu().numpy(), maxes.cpu().numpy()
        return o.cpu().numpy(), ms

    def run_naive_fa2_kernel(self, Q, K, V):
        """The harness's "fa2-naive" run (:374-426): kernels/plain-attn.cu, grid
        B*H*ceil(S/32), 256 threads, VALU-only FA2."""
        import torch

        B, H, S, D = Q.shape
        if D != 64:
            raise ValueError("the plain FA2 wrapper is instantiated for head_dim 64 (plain-attn.cu:286)")
        q, k, v = _to_dev(Q), _to_dev(K), _to_dev(V)
        o = torch.zeros_like(q)
        lse = torch.zeros((B, H, S), device=q.device, dtype=torch.float32)
        shared_mem = (32 * D * 2 + 32 * D * 2 + 32 * 32 + 32 * 3) * 4  # :393-396
        T_r = (S + 31) // 32
        ms = self._timed(lambda: self.forward_fa_naive((B * H * T_r,), (256,), (q, k, v, o, lse, B, H, S),
                                                       shared_mem=shared_mem))
        self.last_lse = lse.cpu().numpy()
        return o.cpu().numpy(), ms

    def run_cuda_naive_kernel(self, Q, K, V):
        import torch

        B, H, S, D = Q.shape
        if D != 64:
            raise ValueError("the naive wrapper is instantiated for head_dim 64 (vanilla-attn.cu:156 in the reference)")
        q, k, v = _to_dev(Q), _to_dev(K), _to_dev(V)
        attn = torch.zeros((B, H, S, S), device=q.device, dtype=torch.float32)
        o = torch.zeros_like(q)
        ms = self._timed(lambda: self.naive_kernel((B * H,), (128,), (q, k, v, o, attn, B, H, S)))
        self.last_p = attn.cpu().numpy()
        return o.cpu().numpy(), ms


def compute_metrics(actual, expected, kernel_time_ms, torch_time_ms, B, H, S, D):
    """The harness's accuracy and speed metrics (test_flash_attention2.py:569-606)."""
    abs_err = np.abs(actual - expected)
    rel = np.where(np.abs(expected) > 1e-8, abs_err / np.maximum(np.abs(expected), 1e-30), 0.0)
    flops = 2 * B * H * S * S * D * 2
    bytes_ = B * H * S * D * 4 * 4
    return {
        "max_abs_error": float(abs_err.max()),
        "mean_abs_error": float(abs_err.mean()),
        "mse": float(((actual - expected) ** 2).mean()),
        "max_rel_error": float(rel.max()),
        "tflops": flops / (kernel_time_ms * 1e-3) / 1e12 if kernel_time_ms > 0 else 0.0,
        "bandwidth_gbps": bytes_ / (kernel_time_ms * 1e-3) / 1e9 if kernel_time_ms > 0 else 0.0,
        "speedup": torch_time_ms / kernel_time_ms if kernel_time_ms > 0 else 0.0,
    }


def passed(metrics, actual, tolerance=1e-3):
    """Pass rule of the harness (:1018-1020): max-abs < tolerance, no NaN/Inf."""
    return metrics["max_abs_error"] < tolerance and np.isfinite(actual).all()
