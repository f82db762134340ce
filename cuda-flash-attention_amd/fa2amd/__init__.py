"""fa2amd -- Python host side of the MI355X-native FA2 forward+backward.

Thin ctypes binding of the C ABI in ``include/fa2_amd.h`` (``lib/libfa2amd.so``,
built by ``make`` in this directory / ``__graft_entry__.build()``).  The product
path is the HIP extension only: if the library is missing or the tensors are not
on a GPU, these functions raise -- there is no CPU fallback.

Tensors are torch fp32, contiguous, [B, H, S, D] (logsumexp / delta [B, H, S]),
exactly the reference's layout (detker/CUDA-Flash-Attention).
``precision`` is ``"fp16"`` (MFMA f16 tiles, fp32 accumulate -- the reference's
``_f16.cu`` variants), ``"fp32"`` (exact fp32 MFMA -- the reference's default) or
``"bf16"`` (MFMA bf16 tiles, fp32 accumulate -- the reference README's "BF16
precision support" improvement, README.md:504-508).
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(_HERE)
LIB_PATH = os.path.join(PKG_ROOT, "lib", "libfa2amd.so")
CLI_PATH = os.path.join(PKG_ROOT, "bin", "FlashAttention")
KERNEL_DIR = os.path.join(PKG_ROOT, "kernels")

FA2_FP16 = 0
FA2_FP32 = 1
FA2_BF16 = 2
_PRECISION = {"fp16": FA2_FP16, "fp32": FA2_FP32, "bf16": FA2_BF16,
              FA2_FP16: FA2_FP16, FA2_FP32: FA2_FP32, FA2_BF16: FA2_BF16}
SUPPORTED_HEAD_DIMS = (32, 64, 128)

# exported symbols of include/fa2_amd.h (checked by tests/test_capi_symbols.py)
C_SYMBOLS = (
    "fa2_forward", "fa2_delta", "fa2_backward", "fa2_backward_dkdv",
    "fa2_backward_dq", "fa2_backward_dq_delta", "fa2_naive_forward", "fa2_fa1_forward",
    "fa2_forward_host", "fa2_backward_host", "fa2_host_release", "fa2_shard_range", "fa2_tune_set", "fa2_tune_get", "fa2_last_error",
    "fa2_version", "fa2_build_id", "fa2_device_count",
)
# launch-plan overrides fa2_tune_set accepts (include/fa2_amd.h)
KNOBS = ("FWD_HS", "FWD_WAVES", "FWD_KS", "FWD_NKB", "DKDV_WAVES", "DKDV_QS", "DKDV_HS", "DQ_WAVES", "DQ_KS", "DQ_HS",
         "BWD_FUSED", "BWD_FUSED_DELTA", "BWD_FQS", "BWD_FKS", "BWD_FNW", "HOST_SHARDS_ON_DEVICE0", "HOST_CHUNKS",
         "FWD_SPLIT", "BWD_SPLIT")


class FA2Error(RuntimeError):
    """A non-zero return code of the C ABI (message from fa2_last_error)."""


_lib = None


def build(jobs: int = 8) -> str:
    """Compile the HIP extension in-tree (hipcc, gfx950)."""
    import subprocess

    subprocess.run(["make", "-s", f"-j{jobs}", "-C", PKG_ROOT], check=True)
    return LIB_PATH


_libs = {}


def use_library(path: str):
    """Switch the active extension to another build of the same C ABI (tools/kbench.py
    A/B's compiler-flag variants in one process this way)."""
    global _lib
    _lib = _libs.get(path) or _load(path)
    _libs[path] = _lib
    return _lib


def lib():
    """Load lib/libfa2amd.so (raises FA2Error if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise FA2Error(f"HIP extension not built: {LIB_PATH} is missing (run __graft_entry__.build())")
    _lib = _load(LIB_PATH)
    return _lib


def _load(path):
    L = ctypes.CDLL(path)
    P, I, V = ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p
    FP = ctypes.POINTER(ctypes.c_float)
    sig = {
        "fa2_forward": [P] * 5 + [I] * 5 + [V],
        "fa2_delta": [P] * 3 + [I] * 4 + [V],
        "fa2_backward": [P] * 10 + [I] * 5 + [V],
        "fa2_backward_dkdv": [P] * 8 + [I] * 4 + [V],
        "fa2_backward_dq": [P] * 7 + [I] * 4 + [V],
        "fa2_backward_dq_delta": [P] * 8 + [I] * 4 + [V],
        "fa2_naive_forward": [P] * 6 + [I] * 4 + [V],
        "fa2_fa1_forward": [P] * 6 + [I] * 4 + [V],
        "fa2_forward_host": [P] * 5 + [I] * 6 + [FP],
        "fa2_backward_host": [P] * 9 + [I] * 6 + [FP],
        "fa2_host_release": [],
        "fa2_shard_range": [I, I, I, ctypes.POINTER(I), ctypes.POINTER(I)],
        "fa2_tune_set": [ctypes.c_char_p, I],
        "fa2_tune_get": [ctypes.c_char_p, ctypes.POINTER(I)],
        "fa2_last_error": [],
        "fa2_version": [],
        "fa2_build_id": [],
        "fa2_device_count": [],
    }
    for name, args in sig.items():
        if path != LIB_PATH and not hasattr(L, name):
            continue  # an older build A/B'd by tools/kbench.py may lack newer entry points
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = ctypes.c_char_p if name in ("fa2_last_error", "fa2_build_id") else I
    return L


def _check(rc: int):
    if rc != 0:
        raise FA2Error(lib().fa2_last_error().decode() or f"fa2 error {rc}")


def version() -> int:
    return lib().fa2_version()


def build_id() -> str:
    """Hash of the sources and flags the loaded library was built from."""
    L = lib()
    return L.fa2_build_id().decode() if hasattr(L, "fa2_build_id") else "unknown"


def tune_set(knob, value: int = 0):
    """Launch-plan override (tests and tools only; fa2_tune_set): ``tune_set(None)``
    clears every override.  Nothing is read from the environment."""
    L = lib()
    if knob is None and not hasattr(L, "fa2_tune_set"):
        return  # an older build (tools/kbench.py A/B) has no overrides to clear
    _check(L.fa2_tune_set(None if knob is None else knob.encode(), int(value)))


def tune_get(knob):
    """The override set for ``knob`` (fa2_tune_get), or None when it has none."""
    v = ctypes.c_int(0)
    rc = lib().fa2_tune_get(knob.encode(), ctypes.byref(v))
    if rc < 0:
        _check(rc)
    return v.value if rc == 1 else None


class tuned:
    """``with fa2amd.tuned(DKDV_QS=2, DKDV_WAVES=8): ...`` -- overrides for the block;
    on exit every override is back to what it was before the block (nested blocks and
    overrides set outside keep their values)."""

    def __init__(self, **knobs):
        self.knobs = knobs
        self.saved = None

    def __enter__(self):
        self.saved = {k: tune_get(k) for k in KNOBS}
        for k, v in self.knobs.items():
            tune_set(k, v)
        return self

    def __exit__(self, *exc):
        tune_set(None)
        for k, v in self.saved.items():
            if v is not None:
                tune_set(k, v)
        return False


def shard_range(total_heads: int, shards: int, index: int):
    """Contiguous balanced head range of shard ``index`` (same rule as the C ABI)."""
    q, r = divmod(total_heads, shards)
    first = index * q + min(index, r)
    return first, q + (1 if index < r else 0)


# ---------------------------------------------------------------------------
# device-tensor API (torch)
# ---------------------------------------------------------------------------
def _dev(t, name, shape=None, device=None):
    """Pointer of a contiguous fp32 GPU tensor, after checking its shape and that it
    lives on `device` (the kernels read and write exactly B*H*S*D / B*H*S elements of
    every pointer: a short or foreign tensor would be read out of bounds)."""
    import torch

    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor")
    if t.dtype != torch.float32:
        raise TypeError(f"{name} must be float32")
    if shape is not None and tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name} has shape {tuple(t.shape)}, expected {tuple(shape)}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    if not t.is_cuda:
        raise FA2Error(f"{name} must be on a GPU (no CPU fallback in the product path)")
    if device is not None and t.device != device:
        raise ValueError(f"{name} is on {t.device}, expected {device}")
    return t.data_ptr()


def _ptrs(named, B, H, S, D, device):
    """[(tensor, name, kind)] -> pointers; kind 4 = [B,H,S,D], 3 = [B,H,S].

    The same checks as `_dev`, first as one cheap conjunction per tensor (the host cost
    of a call bounds small launches: 10 tensors took 6.2 us through `_dev` on the GPU
    box, tools/host_overhead.py); any tensor that fails it goes through `_dev`, which
    raises the specific error."""
    import torch

    s4, s3 = (B, H, S, D), (B, H, S)
    idx = device.index if device.type == "cuda" else None
    f32, T = torch.float32, torch.Tensor
    out = []
    for t, n, kind in named:
        shp = s4 if kind == 4 else s3
        if idx is not None and type(t) is T and t.dtype is f32 and t.get_device() == idx and t.shape == shp \
                and t.is_contiguous():
            out.append(t.data_ptr())
        else:
            out.append(_dev(t, n, shp, device))
    return out


def _stream(stream, device):
    import torch

    if stream is None:
        idx = device.index if device.index is not None else torch.cuda.current_device()
        raw = getattr(torch._C, "_cuda_getCurrentRawStream", None)
        if raw is not None:  # the current stream's handle without building a Stream object
            return ctypes.c_void_p(raw(idx))
        stream = torch.cuda.current_stream(device)
    return ctypes.c_void_p(stream.cuda_stream)


def _shape(q):
    if q.dim() != 4:
        raise ValueError("expected [B, H, S, D]")
    B, H, S, D = q.shape
    if D not in SUPPORTED_HEAD_DIMS:
        raise ValueError(f"head_dim {D} not in {SUPPORTED_HEAD_DIMS}")
    return B, H, S, D


def forward(q, k, v, precision="fp16", out=None, lse=None, stream=None):
    """O, LSE = FA2 forward.  Replaces the reference's fwd kernel launch."""
    import torch

    B, H, S, D = _shape(q)
    out = torch.empty_like(q) if out is None else out
    lse = torch.empty((B, H, S), device=q.device, dtype=torch.float32) if lse is None else lse
    ptrs = _ptrs(((q, "q", 4), (k, "k", 4), (v, "v", 4), (out, "out", 4), (lse, "lse", 3)), B, H, S, D, q.device)
    _check(lib().fa2_forward(*ptrs, B, H, S, D, _PRECISION[precision], _stream(stream, q.device)))
    return out, lse


def delta(dout, o, out=None, stream=None):
    import torch

    B, H, S, D = _shape(o)
    out = torch.empty((B, H, S), device=o.device, dtype=torch.float32) if out is None else out
    ptrs = _ptrs(((dout, "dout", 4), (o, "o", 4), (out, "delta", 3)), B, H, S, D, o.device)
    _check(lib().fa2_delta(*ptrs, B, H, S, D, _stream(stream, o.device)))
    return out


def backward(q, k, v, o, dout, lse, precision="fp16", dq=None, dk=None, dv=None, delta_buf=None, stream=None):
    """dQ, dK, dV = FA2 backward (Δ computed internally into ``delta_buf``)."""
    import torch

    B, H, S, D = _shape(q)
    dq = torch.empty_like(q) if dq is None else dq
    dk = torch.empty_like(q) if dk is None else dk
    dv = torch.empty_like(q) if dv is None else dv
    delta_buf = torch.empty((B, H, S), device=q.device, dtype=torch.float32) if delta_buf is None else delta_buf
    ptrs = _ptrs(((q, "q", 4), (k, "k", 4), (v, "v", 4), (o, "o", 4), (dout, "dout", 4), (lse, "lse", 3),
                  (delta_buf, "delta", 3), (dq, "dq", 4), (dk, "dk", 4), (dv, "dv", 4)), B, H, S, D, q.device)
    _check(lib().fa2_backward(*ptrs, B, H, S, D, _PRECISION[precision], _stream(stream, q.device)))
    return dq, dk, dv


def backward_dkdv(q, k, v, dout, lse, delta_buf, dk, dv, stream=None):
    B, H, S, D = _shape(q)
    ptrs = _ptrs(((q, "q", 4), (k, "k", 4), (v, "v", 4), (dout, "dout", 4), (lse, "lse", 3), (delta_buf, "delta", 3),
                  (dk, "dk", 4), (dv, "dv", 4)), B, H, S, D, q.device)
    _check(lib().fa2_backward_dkdv(*ptrs, B, H, S, D, _stream(stream, q.device)))


def backward_dq(q, k, v, dout, lse, delta_buf, dq, stream=None):
    B, H, S, D = _shape(q)
    ptrs = _ptrs(((q, "q", 4), (k, "k", 4), (v, "v", 4), (dout, "dout", 4), (lse, "lse", 3), (delta_buf, "delta", 3),
                  (dq, "dq", 4)), B, H, S, D, q.device)
    _check(lib().fa2_backward_dq(*ptrs, B, H, S, D, _stream(stream, q.device)))


def backward_dq_delta(q, k, v, o, dout, lse, delta_buf, dq, stream=None):
    """dQ with Δ = rowsum(dO * O) computed in the same kernel and written to delta_buf."""
    B, H, S, D = _shape(q)
    ptrs = _ptrs(((q, "q", 4), (k, "k", 4), (v, "v", 4), (o, "o", 4), (dout, "dout", 4), (lse, "lse", 3),
                  (delta_buf, "delta", 3), (dq, "dq", 4)), B, H, S, D, q.device)
    _check(lib().fa2_backward_dq_delta(*ptrs, B, H, S, D, _stream(stream, q.device)))


def naive_forward(q, k, v, out=None, lse=None, scores=None, stream=None):
    """(O, LSE, P) of the naive baseline (the reference's vanilla attention, CLI
    method ``naive``): the [B, H, S, S] score matrix is materialised (``scores``
    ends holding P).  fp32 only, forward only, as in the reference."""
    import torch

    B, H, S, D = _shape(q)
    out = torch.empty_like(q) if out is None else out
    lse = torch.empty((B, H, S), device=q.device, dtype=torch.float32) if lse is None else lse
    scores = torch.empty((B, H, S, S), device=q.device, dtype=torch.float32) if scores is None else scores
    ptrs = _ptrs(((q, "q", 4), (k, "k", 4), (v, "v", 4), (out, "out", 4), (lse, "lse", 3)), B, H, S, D, q.device)
    ptrs.append(_dev(scores, "scores", (B, H, S, S), q.device))
    _check(lib().fa2_naive_forward(*ptrs, B, H, S, D, _stream(stream, q.device)))
    return out, lse, scores


def fa1_forward(q, k, v, out=None, l=None, m=None, stream=None):
    """(O, l, m) of the FlashAttention-1 baseline (CLI method ``fa1``): l is the row
    sum relative to m (the reference's ``logsumexp`` output), so LSE = m + ln l."""
    import torch

    B, H, S, D = _shape(q)
    out = torch.empty_like(q) if out is None else out
    l = torch.empty((B, H, S), device=q.device, dtype=torch.float32) if l is None else l
    m = torch.empty((B, H, S), device=q.device, dtype=torch.float32) if m is None else m
    ptrs = _ptrs(((q, "q", 4), (k, "k", 4), (v, "v", 4), (out, "out", 4), (l, "l", 3), (m, "m", 3)), B, H, S, D,
                 q.device)
    _check(lib().fa2_fa1_forward(*ptrs, B, H, S, D, _stream(stream, q.device)))
    return out, l, m


# ---------------------------------------------------------------------------
# host-array API (numpy): the reference host functions' semantics
# ---------------------------------------------------------------------------
def _np(a, name, shape=None):
    """Pointer of a C-contiguous float32 array of exactly `shape` (the library copies
    B*H*S*D / B*H*S floats from every host pointer)."""
    import numpy as np

    if not (isinstance(a, np.ndarray) and a.dtype == np.float32 and a.flags.c_contiguous):
        raise TypeError(f"{name} must be a C-contiguous float32 numpy array")
    if shape is not None and a.shape != tuple(shape):
        raise ValueError(f"{name} has shape {a.shape}, expected {tuple(shape)}")
    return a.ctypes.data_as(ctypes.c_void_p)


def _host_shape(q):
    import numpy as np

    if not isinstance(q, np.ndarray) or q.ndim != 4:
        raise ValueError("expected q as a [B, H, S, D] numpy array")
    return q.shape


def forward_host(q, k, v, precision="fp32", num_devices=1, out=None, lse=None):
    """(O, LSE, kernel_ms) from host arrays: host_flash_attention2_forward[_fp16] semantics.
    ``out`` / ``lse``: caller-owned result arrays (reused, as a caller looping over
    batches would; fresh ones are allocated otherwise)."""
    import numpy as np

    B, H, S, D = _host_shape(q)
    o = np.empty_like(q) if out is None else out
    lse = np.empty((B, H, S), np.float32) if lse is None else lse
    ms = ctypes.c_float(0.0)
    _check(lib().fa2_forward_host(_np(q, "q"), _np(k, "k", q.shape), _np(v, "v", q.shape), _np(o, "o", q.shape),
                                  _np(lse, "lse", (B, H, S)), B, H, S, D, _PRECISION[precision], num_devices,
                                  ctypes.byref(ms)))
    return o, lse, ms.value


def backward_host(q, k, v, o, dout, lse, precision="fp32", num_devices=1, dq=None, dk=None, dv=None):
    """(dQ, dK, dV, kernel_ms) from host arrays: host_flash_attention2_backward[_fp16]
    semantics (``dq`` / ``dk`` / ``dv``: caller-owned result arrays, optional)."""
    import numpy as np

    B, H, S, D = _host_shape(q)
    dq = np.empty_like(q) if dq is None else dq
    dk = np.empty_like(q) if dk is None else dk
    dv = np.empty_like(q) if dv is None else dv
    ms = ctypes.c_float(0.0)
    _check(lib().fa2_backward_host(_np(q, "q"), _np(k, "k", q.shape), _np(v, "v", q.shape), _np(o, "o", q.shape),
                                   _np(dout, "dout", q.shape), _np(lse, "lse", (B, H, S)), _np(dq, "dq", q.shape),
                                   _np(dk, "dk", q.shape), _np(dv, "dv", q.shape),
                                   B, H, S, D, _PRECISION[precision], num_devices, ctypes.byref(ms)))
    return dq, dk, dv, ms.value


def host_release():
    """Free the device scratch the host-pointer API keeps between calls."""
    _check(lib().fa2_host_release())
