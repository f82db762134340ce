"""ctypes binding of oracle/fa2_oracle.c (TEST INFRASTRUCTURE ONLY -- see fa2_oracle.py)."""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle_fa2.so")
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        lib = ctypes.CDLL(_LIB_PATH)
        fp = ctypes.POINTER(ctypes.c_float)
        i = ctypes.c_int
        lib.oracle_fa2_forward.argtypes = [fp] * 5 + [i] * 5
        lib.oracle_fa2_backward.argtypes = [fp] * 9 + [i] * 5
        lib.oracle_fa2_delta.argtypes = [fp] * 3 + [i] * 4
        lib.oracle_fa2_forward.restype = i
        lib.oracle_fa2_backward.restype = i
        _lib = lib
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def _c(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def forward(q, k, v, nthreads: int = 1):
    q, k, v = _c(q), _c(k), _c(v)
    B, H, S, D = q.shape
    o = np.empty_like(q)
    lse = np.empty((B, H, S), np.float32)
    rc = _load().oracle_fa2_forward(_p(q), _p(k), _p(v), _p(o), _p(lse), B, H, S, D, nthreads)
    if rc != 0:
        raise ValueError("oracle_fa2_forward rejected its arguments")
    return o, lse


def backward(q, k, v, o, do, lse, nthreads: int = 1):
    q, k, v, o, do, lse = (_c(x) for x in (q, k, v, o, do, lse))
    B, H, S, D = q.shape
    dq, dk, dv = np.empty_like(q), np.empty_like(q), np.empty_like(q)
    rc = _load().oracle_fa2_backward(_p(q), _p(k), _p(v), _p(o), _p(do), _p(lse),
                                     _p(dq), _p(dk), _p(dv), B, H, S, D, nthreads)
    if rc != 0:
        raise ValueError("oracle_fa2_backward rejected its arguments")
    return dq, dk, dv


def delta(do, o):
    do, o = _c(do), _c(o)
    B, H, S, D = o.shape
    out = np.empty((B, H, S), np.float32)
    _load().oracle_fa2_delta(_p(do), _p(o), _p(out), B, H, S, D)
    return out
