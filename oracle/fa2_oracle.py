"""CPU oracle for the FA2 forward+backward hot path.

TEST INFRASTRUCTURE ONLY.  This module is the *checker*: it may be imported by
``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
``bench.py`` -- never by the product path (``cuda-flash-attention_amd/``), which
must fail loudly when its HIP extension is missing.

It restates, in numpy, the reference's own oracle and data generators
(detker/CUDA-Flash-Attention, mounted read-only at /root/reference):

* inputs, harness distribution -- ``FlashAttention2Tester.generate_test_data``
  (test_flash_attention2.py:177-195): ``torch.manual_seed(seed)`` then
  ``torch.rand`` U[0,1) fp32 for Q, K, V in that order.  (torch is used here
  only as the RNG so the bytes match the reference; the arithmetic is numpy.)
* inputs, CLI distribution -- ``generate_test_data`` (generate_test_data.py:6-33):
  ``np.random.seed(seed)`` then ``randn`` for Q, K, V.
* forward -- ``compute_reference`` (test_flash_attention2.py:197-208):
  scores = Q Kᵀ / √D, softmax over the key axis, times V.
* logsumexp -- test_flash_attention2.py:917-921 (natural log, max-shifted),
  the same quantity the kernels write (kernel_fa2_optimized.cu:341-343).
* backward -- ``compute_reference_backward`` (test_flash_attention2.py:220-232)
  is autograd of the forward; its closed form is restated here:
  dV = Pᵀ dO, dP = dO Vᵀ, Δ = rowsum(dO∘O) (f-attn2-backward.cu:341-380),
  dS = P∘(dP − Δ), dQ = dS K / √D, dK = dSᵀ Q / √D (f-attn2-backward.cu:218-323).
* tile emulator -- the FA2 online-softmax recurrence over 32×32 tiles exactly
  as kernel_fa2_optimized.cu:89-346 orders it, with an optional fp16 storage
  rounding point set that mirrors kernel_fa2_optimized_f16.cu (a3 in SURVEY §8).

Parity pinning: ``tests/test_oracle_golden.py`` checks every function here
against the fixtures in ``tests/golden/`` that ``tests/golden/make_golden.py``
produced by importing the reference harness itself.
"""
from __future__ import annotations

import numpy as np

__all__ = [
    "harness_inputs",
    "cli_inputs",
    "attention_forward",
    "attention_backward",
    "delta",
    "attention_forward_tiled",
    "fwd_flops",
    "bwd_flops",
    "fwd_bytes",
    "bwd_bytes",
]


# --------------------------------------------------------------------------
# input generators (bit-identical to the reference's)
# --------------------------------------------------------------------------
def harness_inputs(B: int, H: int, S: int, D: int, seed: int = 42):
    """Q, K, V as ``test_flash_attention2.py:177-195`` draws them (float32)."""
    import torch  # RNG only: torch.rand's bit stream is the reference's input

    torch.manual_seed(seed)
    np.random.seed(seed)
    q = torch.rand(B, H, S, D, dtype=torch.float32).numpy()
    k = torch.rand(B, H, S, D, dtype=torch.float32).numpy()
    v = torch.rand(B, H, S, D, dtype=torch.float32).numpy()
    return q, k, v


def cli_inputs(B: int, H: int, S: int, D: int, seed: int = 42):
    """Q, K, V as ``generate_test_data.py:10,27-33`` draws them (float32)."""
    rs = np.random.RandomState(seed)  # same stream as np.random.seed(seed)
    shape = (B, H, S, D)
    q = rs.randn(*shape).astype(np.float32)
    k = rs.randn(*shape).astype(np.float32)
    v = rs.randn(*shape).astype(np.float32)
    return q, k, v


# --------------------------------------------------------------------------
# math oracle (float64 internally, float32 out)
# --------------------------------------------------------------------------
def _scores(q, k):
    d = q.shape[-1]
    return np.matmul(q.astype(np.float64), np.swapaxes(k.astype(np.float64), -1, -2)) / np.sqrt(d)


def attention_forward(q, k, v):
    """(O, LSE) for fp32 [B,H,S,D] inputs; test_flash_attention2.py:197-208, 917-921."""
    s = _scores(q, k)
    m = s.max(axis=-1, keepdims=True)
    e = np.exp(s - m)
    l = e.sum(axis=-1, keepdims=True)
    p = e / l
    o = np.matmul(p, v.astype(np.float64))
    lse = (m + np.log(l))[..., 0]
    return o.astype(np.float32), lse.astype(np.float32)


def delta(do, o):
    """Δ_i = Σ_d dO_id · O_id  (D_computation_reduction_kernel, f-attn2-backward.cu:341-380)."""
    return (do.astype(np.float64) * o.astype(np.float64)).sum(-1).astype(np.float32)


def attention_backward(q, k, v, do):
    """(dQ, dK, dV, Δ) = autograd of ``compute_reference`` for upstream grad dO.

    Closed form of test_flash_attention2.py:220-232 (which uses dO = ones);
    the loop structure it replaces is f-attn2-backward.cu:119-338.
    """
    d = q.shape[-1]
    s = _scores(q, k)
    m = s.max(axis=-1, keepdims=True)
    e = np.exp(s - m)
    p = e / e.sum(axis=-1, keepdims=True)
    q64, k64, v64, do64 = (x.astype(np.float64) for x in (q, k, v, do))
    o = np.matmul(p, v64)
    dv = np.matmul(np.swapaxes(p, -1, -2), do64)
    dp = np.matmul(do64, np.swapaxes(v64, -1, -2))
    dl = (do64 * o).sum(-1, keepdims=True)
    ds = p * (dp - dl)
    dq = np.matmul(ds, k64) / np.sqrt(d)
    dk = np.matmul(np.swapaxes(ds, -1, -2), q64) / np.sqrt(d)
    return (dq.astype(np.float32), dk.astype(np.float32), dv.astype(np.float32),
            dl[..., 0].astype(np.float32))


# --------------------------------------------------------------------------
# tile-faithful emulator of the reference FA2 forward
# --------------------------------------------------------------------------
def attention_forward_tiled(q, k, v, br: int = 32, bc: int = 32, storage=np.float32):
    """FA2 forward with the reference kernel's tiling and rounding points.

    Follows kernel_fa2_optimized.cu:60-346: per 32-row Q tile, loop over 32-col
    KV tiles (``:89``): S = QKᵀ/√D (``:187``), -FLT_MAX for cols >= S
    (``:183-184``), m_new = max(m, rowmax) (``:217-226``), P = exp(S - m_new)
    (``:228-233``), l = e^{m-m_new}·l + rowsum(P) (``:249-253``),
    O = O·e^{m-m_new} + P V (``:295-319``); O/l and LSE = ln l + m (``:336-343``).
    ``storage=np.float16`` rounds Q, K, V, S/P, O, m, l where
    kernel_fa2_optimized_f16.cu stores them as __half; the
    products and sums themselves stay fp32 as in that kernel.
    """
    B, H, S, D = q.shape
    f32 = np.float32
    rnd = (lambda x: x.astype(storage).astype(f32)) if storage is not np.float32 else (lambda x: x.astype(f32))
    qs, ks, vs = rnd(q), rnd(k), rnd(v)
    o_out = np.zeros((B, H, S, D), f32)
    lse_out = np.zeros((B, H, S), f32)
    scale = f32(np.sqrt(f32(D)))
    neg = f32(-3.402823466e38)
    for b in range(B):
        for h in range(H):
            for r0 in range(0, S, br):
                rows = slice(r0, min(r0 + br, S))
                qt = qs[b, h, rows]
                n = qt.shape[0]
                m = np.full(n, neg, f32)
                l = np.zeros(n, f32)
                o = np.zeros((n, D), f32)
                for c0 in range(0, S, bc):
                    cols = slice(c0, min(c0 + bc, S))
                    kt, vt = ks[b, h, cols], vs[b, h, cols]
                    st = rnd((qt @ kt.T).astype(f32) / scale)
                    rowmax = st.max(axis=1)
                    m_new = rnd(np.maximum(m, rowmax))
                    coeff = rnd(np.exp(m - m_new).astype(f32))
                    p = rnd(np.exp(st - m_new[:, None]).astype(f32))
                    l = rnd(coeff * l + p.sum(axis=1, dtype=f32))
                    o = rnd(o * coeff[:, None] + (p @ vt).astype(f32))
                    m = m_new
                o_out[b, h, rows] = o / l[:, None]
                lse_out[b, h, rows] = np.log(l) + m
    return o_out, lse_out


# --------------------------------------------------------------------------
# algorithmic work
# --------------------------------------------------------------------------
def fwd_flops(B, H, S, D):
    return 4.0 * B * H * S * S * D


def bwd_flops(B, H, S, D):
    return 10.0 * B * H * S * S * D


def fwd_bytes(B, H, S, D):
    """read Q,K,V + write O (fp32) + write LSE."""
    return 16.0 * B * H * S * D + 4.0 * B * H * S


def bwd_bytes(B, H, S, D):
    """read Q,K,V,O,dO + LSE, write dQ,dK,dV (fp32)."""
    return 32.0 * B * H * S * D + 4.0 * B * H * S
