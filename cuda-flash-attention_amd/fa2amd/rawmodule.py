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


def _libdir():
    """Directory of the HIP runtime to bind.  Once torch is imported its bundled
    libamdhip64 / libhsa-runtime64 are the process's HIP runtime; a second copy
    from /opt/rocm would not resolve against them (undefined hsa_* symbols), so
    bind torch's copies then, and /opt/rocm's otherwise."""
    import sys

    t = sys.modules.get("torch")
    if t is not None:
        d = os.path.join(os.path.dirname(t.__file__), "lib")
        if os.path.exists(os.path.join(d, "libamdhip64.so")):
            return d
    return os.path.join(ROCM, "lib")


def _hiprtc():
    global _rtc
    if _rtc is None:
        _rtc = ctypes.CDLL(os.path.join(_libdir(), "libhiprtc.so"))
    return _rtc


def _hipapi():
    global _hip
    if _hip is None:
        _hip = ctypes.CDLL(os.path.join(_libdir(), "libamdhip64.so"))
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


MAX_LDS_BYTES = 160 * 1024  # per workgroup on gfx950 (MI355X_MICROARCH.md, LDS per CU)


def static_lds_bytes(code_object: bytes) -> dict:
    """{kernel: group_segment_fixed_size} from the code object's AMDGPU metadata note."""
    import subprocess
    import tempfile

    readelf = os.path.join(ROCM, "lib", "llvm", "bin", "llvm-readelf")
    with tempfile.NamedTemporaryFile(suffix=".co") as f:
        f.write(code_object)
        f.flush()
        out = subprocess.run([readelf, "--notes", f.name], capture_output=True, text=True, check=True).stdout
    sizes, pending = {}, None
    for line in out.splitlines():
        line = line.strip()
        if line.startswith(".group_segment_fixed_size:"):
            pending = int(line.split(":")[1])
        elif line.startswith(".name:") and pending is not None:
            sizes[line.split(":", 1)[1].strip()] = pending
            pending = None
    return sizes


class RawFunction:
    def __init__(self, fn, name="", static_lds=0):
        self._fn = fn
        self.name = name
        self.static_lds = static_lds

    def __call__(self, grid, block, args, shared_mem=0, stream=None):
        """Launch like ``cupy.RawKernel.__call__``: tensors by data pointer, ints as int64."""
        import torch

        if self.static_lds + shared_mem > MAX_LDS_BYTES:
            raise HipError(f"{self.name}: {self.static_lds} B static + {shared_mem} B dynamic LDS exceeds "
                           f"the {MAX_LDS_BYTES} B a workgroup may own")
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
        self.static_lds = static_lds_bytes(self.code_object)
        self._mod = ctypes.c_void_p()
        _chk(_hipapi().hipModuleLoadData(ctypes.byref(self._mod), self.code_object), "hipModuleLoadData")

    def get_function(self, name: str) -> RawFunction:
        fn = ctypes.c_void_p()
        _chk(_hipapi().hipModuleGetFunction(ctypes.byref(fn), self._mod, name.encode()), "hipModuleGetFunction")
        return RawFunction(fn, name, self.static_lds.get(name, 0))


def load_kernel_source(filename: str) -> str:
    """Text of one of this package's reference-named kernel files (kernels/<filename>)."""
    from . import KERNEL_DIR

    with open(os.path.join(KERNEL_DIR, filename)) as f:
        return f.read()
