"""ctypes loader for oracle/_build/liboracle.so (TEST INFRASTRUCTURE)."""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = ctypes.CDLL(_SO)
        i64, i32, p, d = ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p, ctypes.c_double
        L.orc_fedavg_ref.argtypes = [p, i64, p, p, i32, i64, p]
        L.orc_dequant_rows.argtypes = [p, i64, i64, p, p, p]
        L.orc_sign_direction.argtypes = [p, p, p, i64, d, d, i32, i32]
        L.orc_sign_apply.argtypes = [p, p, i64, d, d]
        L.orc_fastdiv_check.argtypes = [ctypes.c_float]
        L.orc_fastdiv_check.restype = i64
        _lib = L
    return _lib


def ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def fedavg_ref(U, n, order):
    U = np.ascontiguousarray(U, np.float32)
    order = np.ascontiguousarray(order, np.int32)
    n = np.ascontiguousarray(n, np.int64)
    out = np.empty(U.shape[1], np.float32)
    lib().orc_fedavg_ref(ptr(U), U.shape[1], ptr(order), ptr(n), len(order), U.shape[1], ptr(out))
    return out


def dequant_rows(q, scale, zp):
    q = np.ascontiguousarray(q, np.int32)
    C = q.shape[0]
    row = int(np.prod(q.shape[1:])) if q.ndim > 1 else 1
    out = np.empty(q.shape, np.float32)
    lib().orc_dequant_rows(ptr(q), C, row, ptr(np.ascontiguousarray(scale, np.float64)),
                           ptr(np.ascontiguousarray(zp, np.int64)), ptr(out))
    return out


def sign_direction(g, buf, first, momentum, dampening, nesterov):
    g = np.ascontiguousarray(g, np.float32)
    buf = np.array(buf if buf is not None else np.zeros_like(g), np.float32)
    d = np.empty_like(g)
    lib().orc_sign_direction(ptr(g), ptr(buf), ptr(d), g.size, momentum, dampening,
                             int(bool(nesterov)), int(bool(first)))
    return d, buf


def sign_apply(p, vote, lr, wd):
    p = np.array(p, np.float32)
    lib().orc_sign_apply(ptr(p), ptr(np.ascontiguousarray(vote, np.float32)), p.size, lr, wd)
    return p


def fastdiv_check(b):
    return int(lib().orc_fastdiv_check(float(b)))
