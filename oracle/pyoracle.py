"""ctypes wrapper of oracle/build/libggml_oracle.so -- TEST INFRASTRUCTURE ONLY.

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, always as
the checker / CPU baseline, never as the measured or shipped path.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libggml_oracle.so")

# enum ggml_type values (include/ggml/ggml.h:348-381)
F32, F16, Q4_0, Q8_0, Q4_K, Q5_K, Q8_K = 0, 1, 2, 8, 12, 13, 15
TYPE_NAMES = {F32: "f32", F16: "f16", Q4_0: "q4_0", Q8_0: "q8_0", Q4_K: "q4_K", Q5_K: "q5_K", Q8_K: "q8_K"}
TYPES_BY_NAME = {v: k for k, v in TYPE_NAMES.items()}

_lib = None


def build() -> None:
    subprocess.check_call(["make", "-s", "-C", HERE, "oracle"])


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        vp, i64, sz = ctypes.c_void_p, ctypes.c_int64, ctypes.c_size_t
        L.orc_row_size.argtypes = [ctypes.c_int, i64]
        L.orc_row_size.restype = sz
        L.orc_vec_dot_type.argtypes = [ctypes.c_int]
        L.orc_vec_dot_type.restype = ctypes.c_int
        L.orc_quantize_chunk.argtypes = [ctypes.c_int, vp, vp, i64, i64]
        L.orc_quantize_chunk.restype = sz
        L.orc_quantize_act.argtypes = [ctypes.c_int, vp, vp, i64]
        L.orc_dequantize_row.argtypes = [ctypes.c_int, vp, vp, i64]
        L.orc_vec_dot.argtypes = [ctypes.c_int, ctypes.c_int, vp, vp]
        L.orc_vec_dot.restype = ctypes.c_float
        L.orc_mul_mat.argtypes = [ctypes.c_int, vp, i64, i64, vp, i64, vp, ctypes.c_int]
        L.orc_fp32_to_fp16.argtypes = [ctypes.c_float]
        L.orc_fp32_to_fp16.restype = ctypes.c_uint16
        _lib = L
    return _lib


def _p(a: np.ndarray) -> ctypes.c_void_p:
    return ctypes.c_void_p(a.ctypes.data)


def row_size(t: int, n: int) -> int:
    return int(lib().orc_row_size(t, n))


def vec_dot_type(t: int) -> int:
    return int(lib().orc_vec_dot_type(t))


def quantize(t: int, x: np.ndarray, n_per_row: int) -> np.ndarray:
    x = np.ascontiguousarray(x, dtype=np.float32)
    nrows = x.size // n_per_row
    out = np.empty(nrows * row_size(t, n_per_row), dtype=np.uint8)
    lib().orc_quantize_chunk(t, _p(x), _p(out), nrows, n_per_row)
    return out


def quantize_act(vdt: int, x: np.ndarray, K: int) -> np.ndarray:
    x = np.ascontiguousarray(x, dtype=np.float32)
    cols = x.size // K
    rs = row_size(vdt, K)
    out = np.empty(cols * rs, dtype=np.uint8)
    for c in range(cols):
        lib().orc_quantize_act(vdt, _p(x[c * K:(c + 1) * K]), ctypes.c_void_p(out.ctypes.data + c * rs), K)
    return out


def dequantize(t: int, q: np.ndarray, n: int) -> np.ndarray:
    q = np.ascontiguousarray(q)
    out = np.empty(n, dtype=np.float32)
    lib().orc_dequantize_row(t, _p(q), _p(out), n)
    return out


def mul_mat(t: int, wq: np.ndarray, K: int, N: int, x: np.ndarray, B: int, nthreads: int = 8) -> np.ndarray:
    wq = np.ascontiguousarray(wq)
    x = np.ascontiguousarray(x, dtype=np.float32)
    y = np.empty(N * B, dtype=np.float32)
    lib().orc_mul_mat(t, _p(wq), K, N, _p(x), B, _p(y), nthreads)
    return y
