"""Minimal stand-in for ``cupy.RawModule`` on ROCm: hiprtc + hipModule via ctypes.

The reference harness drives the kernels through
``cp.RawModule(code=<file text>, options=('-std=c++14', '-DCUPY_INLINE_COMPILE'),
name_expressions=...)`` and launches the ``extern "C"`` wrappers with a fixed
geometry (test_flash_attention2.py:113-145, 266-308, 499-559).  CuPy is not
installed in this image, so the tests reproduce that exact contract here:
compile the same source text with hiprtc and the same options (plus the gfx950
target, which cupy-rocm adds for the current device), then launch through
``hipModuleLaunchKernel`` with the harness's grid/block/dynamic-LDS and with
Python ints marshalled as 64-bit values the way CuPy passes them.

``compile_source`` needs no GPU (hiprtc cross-compiles); ``RawModule.get_function``
and launching need one.
"""
from __future__ import annotations

import ctypes
import os
import re

ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HARNESS_OPTIONS = ("-std=c++14", "-DCUPY_INLINE_COMPILE")

_rtc = None
_hip = None


def _hiprtc():
    global _rtc
    if _rtc is None:
        _rtc = ctypes.CDLL(os.path.join(ROCM, "lib", "libhiprtc.so"))
    return _rtc


def _hipapi():
    global _hip
    if _hip is None:
        _hip = ctypes.CDLL(os.path.join(ROCM, "lib", "libamdhip64.so"))
    return _hip


class HipError(RuntimeError):
    pass


def _chk_rtc(rc, what, prog=None):
    if rc != 0:
        log = ""
        if prog is not None:
            n = ctypes.c_size_t(0)
            _hiprtc().hiprtcGetProgramLogSize(prog, ctypes.byref(n))
            buf = ctypes.create_string_buffer(n.value + 1)
            _hiprtc().hiprtcGetProgramLog(prog, buf)
            log = buf.value.decode(errors="replace")
        raise HipError(f"{what} failed (hiprtc {rc})\n{log}")


def _chk(rc, what):
    if rc != 0:
        f = _hipapi().hipGetErrorString
        f.restype = ctypes.c_char_p
        raise HipError(f"{what}: {f(rc).decode()} ({rc})")


def compile_source(code: str, options=HARNESS_OPTIONS, arch: str = "gfx950", name: str = "kernel.cu") -> bytes:
    """hiprtc-compile ``code`` with the harness options; returns the code object."""
    rtc = _hiprtc()
    prog = ctypes.c_void_p()
    _chk_rtc(rtc.hiprtcCreateProgram(ctypes.byref(prog), code.encode(), name.encode(), 0, None, None),
             "hiprtcCreateProgram")
    try:
        opts = list(options) + [f"--offload-arch={arch}"]
        arr = (ctypes.c_char_p * len(opts))(*[o.encode() for o in opts])
        _chk_rtc(rtc.hiprtcCompileProgram(prog, len(opts), arr), "hiprtcCompileProgram", prog)
        n = ctypes.c_size_t(0)
        _chk_rtc(rtc.hiprtcGetCodeSize(prog, ctypes.byref(n)), "hiprtcGetCodeSize")
        buf = ctypes.create_string_buffer(n.value)
        _chk_rtc(rtc.hiprtcGetCode(prog, buf), "hiprtcGetCode")
        return buf.raw
    finally:
        rtc.hiprtcDestroyProgram(ctypes.byref(prog))


def exported_kernels(code_object: bytes):
    """Names of the kernel symbols (``<name>.kd`` descriptors) in a code object."""
    return sorted({m.decode() for m in re.findall(rb"([A-Za-z_][A-Za-z0-9_]*)\.kd\x00", code_object)})


class RawFunction:
    def __init__(self, fn):
        self._fn = fn

    def __call__(self, grid, block, args, shared_mem=0, stream=None):
        """Launch like ``cupy.RawKernel.__call__``: tensors by data pointer, ints as int64."""
        import torch

        storage = []
        for a in args:
            if isinstance(a, torch.Tensor):
                storage.append(ctypes.c_void_p(a.data_ptr()))
            elif isinstance(a, bool):
                raise TypeError("bool kernel args are not part of the harness contract")
            elif isinstance(a, int):
                storage.append(ctypes.c_int64(a))  # CuPy marshals Python int as 64-bit
            elif isinstance(a, float):
                storage.append(ctypes.c_double(a))
            else:
                raise TypeError(f"unsupported kernel arg {type(a)}")
        params = (ctypes.c_void_p * len(storage))(*[ctypes.cast(ctypes.byref(s), ctypes.c_void_p) for s in storage])
        g = tuple(grid) + (1,) * (3 - len(grid))
        b = tuple(block) + (1,) * (3 - len(block))
        st = ctypes.c_void_p(stream.cuda_stream if stream is not None else torch.cuda.current_stream().cuda_stream)
        _chk(_hipapi().hipModuleLaunchKernel(self._fn, ctypes.c_uint(g[0]), ctypes.c_uint(g[1]), ctypes.c_uint(g[2]),
                                             ctypes.c_uint(b[0]), ctypes.c_uint(b[1]), ctypes.c_uint(b[2]),
                                             ctypes.c_uint(shared_mem), st, params, None),
             "hipModuleLaunchKernel")


class RawModule:
    """``cp.RawModule(code=..., options=..., name_expressions=...)`` equivalent."""

    def __init__(self, code: str, options=HARNESS_OPTIONS, name_expressions=(), arch: str = "gfx950"):
        self.code_object = compile_source(code, options, arch)
        missing = [n for n in name_expressions if n not in exported_kernels(self.code_object)]
        if missing:
            raise HipError(f"symbols not exported by the module: {missing}")
        self._mod = ctypes.c_void_p()
        _chk(_hipapi().hipModuleLoadData(ctypes.byref(self._mod), self.code_object), "hipModuleLoadData")

    def get_function(self, name: str) -> RawFunction:
        fn = ctypes.c_void_p()
        _chk(_hipapi().hipModuleGetFunction(ctypes.byref(fn), self._mod, name.encode()), "hipModuleGetFunction")
        return RawFunction(fn)


def load_kernel_source(filename: str) -> str:
    """Text of one of this package's reference-named kernel files (kernels/<filename>)."""
    from . import KERNEL_DIR

    with open(os.path.join(KERNEL_DIR, filename)) as f:
        return f.read()
