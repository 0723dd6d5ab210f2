"""ctypes wrapper of oracle/mt19937.c -- TEST INFRASTRUCTURE ONLY.

A RandomState-like object restating NumPy's legacy MT19937 stream
(randint with masked rejection, polar-method normal).  See mt19937.c.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libmt19937_oracle.so")
_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        u32p = ctypes.POINTER(ctypes.c_uint32)
        L.mto_seed.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
        L.mto_set_state.argtypes = [ctypes.c_void_p, u32p, ctypes.c_int32, ctypes.c_int32, ctypes.c_double]
        L.mto_get_state.argtypes = [ctypes.c_void_p, u32p, ctypes.POINTER(ctypes.c_int32),
                                    ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_double)]
        L.mto_next32.argtypes = [ctypes.c_void_p]
        L.mto_next32.restype = ctypes.c_uint32
        L.mto_randint.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p]
        L.mto_randint.restype = ctypes.c_int
        L.mto_normal.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
        L.mto_state_size.restype = ctypes.c_int64
        _lib = L
    return _lib


class MTOracle:
    """Legacy RandomState restatement (subset used by the SAC hot path)."""

    def __init__(self, seed: int | None = None):
        L = lib()
        self._buf = ctypes.create_string_buffer(int(L.mto_state_size()))
        if seed is not None:
            L.mto_seed(self._buf, ctypes.c_uint32(seed & 0xFFFFFFFF))

    def set_state(self, state):
        """Accepts np.random.RandomState.get_state() tuples."""
        _, key, pos, has_gauss, gauss = state[:5]
        key = np.ascontiguousarray(key, dtype=np.uint32)
        lib().mto_set_state(self._buf, key.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                            int(pos), int(has_gauss), float(gauss))

    def get_state(self):
        key = np.zeros(624, np.uint32)
        pos, hg, g = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_double()
        lib().mto_get_state(self._buf, key.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                            ctypes.byref(pos), ctypes.byref(hg), ctypes.byref(g))
        return ("MT19937", key, pos.value, hg.value, g.value)

    def randint(self, high: int, size: int) -> np.ndarray:
        out = np.empty(int(size), np.int64)
        rc = lib().mto_randint(self._buf, int(high), int(size), out.ctypes.data)
        if rc != 0:
            raise ValueError("high out of range")
        return out

    def normal(self, size) -> np.ndarray:
        n = int(np.prod(size))
        out = np.empty(n, np.float64)
        lib().mto_normal(self._buf, n, out.ctypes.data)
        return out.reshape(size)

    def next32(self) -> int:
        return int(lib().mto_next32(self._buf))
