"""GGUF model files onto the MI355X backend, through the runtime's gguf_* API (csrc/core/gguf.cpp).

`Model(lib, path, backend)` is the loading sequence the reference's GGUF examples use
(examples/magika/main.cpp:92-173, examples/yolo): gguf_init_from_file with no_alloc=true and a
ggml_context for the tensor metadata, one backend buffer for every tensor of that context
(ggml_backend_alloc_ctx_tensors), then each tensor's bytes read from the file at
data_offset + tensor_offset and uploaded with ggml_backend_tensor_set. `write(...)` writes a GGUF
file from numpy arrays (key/values + tensors), the way the reference's converters do through
gguf_add_tensor / gguf_write_to_file.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import ggml as G

GGUF_TYPE = dict(u8=0, i8=1, u16=2, i16=3, u32=4, i32=5, f32=6, bool=7, str=8, arr=9, u64=10, i64=11, f64=12)
_NP = {0: np.uint8, 1: np.int8, 2: np.uint16, 3: np.int16, 4: np.uint32, 5: np.int32, 6: np.float32, 7: np.bool_,
       10: np.uint64, 11: np.int64, 12: np.float64}
_GETTER = {0: "u8", 1: "i8", 2: "u16", 3: "i16", 4: "u32", 5: "i32", 6: "f32", 7: "bool", 10: "u64", 11: "i64", 12: "f64"}


class Model:
    """Tensors of a GGUF file resident in one backend buffer; `kv` holds the key/values."""

    def __init__(self, lib: G.Lib, path: str, backend):
        self.lib = lib
        self.buffer = self.ctx = None
        meta = ctypes.c_void_p()
        self.gguf = lib.gguf_init_from_file(path.encode(), G.gguf_init_params(True, ctypes.pointer(meta)))
        if not self.gguf:
            raise RuntimeError(f"gguf_init_from_file({path}) failed")
        self.ctx = meta.value
        self.buffer = lib.ggml_backend_alloc_ctx_tensors(self.ctx, backend)
        if not self.buffer:
            self.free()
            raise RuntimeError("backend buffer allocation failed")
        self.kv = read_kv(lib, self.gguf)
        self.tensors = {}
        base = lib.gguf_get_data_offset(self.gguf)
        with open(path, "rb") as f:
            for i in range(lib.gguf_get_n_tensors(self.gguf)):
                name = lib.gguf_get_tensor_name(self.gguf, i)
                t = lib.ggml_get_tensor(self.ctx, name)
                n = lib.ggml_nbytes(t)
                f.seek(base + lib.gguf_get_tensor_offset(self.gguf, i))
                buf = np.frombuffer(f.read(n), dtype=np.uint8)
                if buf.size != n:
                    self.free()
                    raise RuntimeError(f"{path}: truncated data for tensor {name!r}")
                lib.ggml_backend_tensor_set(t, buf.ctypes.data, 0, n)
                self.tensors[name.decode()] = t

    def free(self):
        if self.buffer:
            self.lib.ggml_backend_buffer_free(self.buffer)
            self.buffer = None
        if self.ctx:
            self.lib.ggml_free(self.ctx)
            self.ctx = None
        if self.gguf:
            self.lib.gguf_free(self.gguf)
            self.gguf = None


def read_kv(lib: G.Lib, g) -> dict:
    """All key/values of a gguf_context as Python values (arrays as numpy / lists of bytes)."""
    out = {}
    for i in range(lib.gguf_get_n_kv(g)):
        key = lib.gguf_get_key(g, i).decode()
        t = lib.gguf_get_kv_type(g, i)
        if t == GGUF_TYPE["str"]:
            out[key] = lib.gguf_get_val_str(g, i)
        elif t == GGUF_TYPE["arr"]:
            at, n = lib.gguf_get_arr_type(g, i), lib.gguf_get_arr_n(g, i)
            if at == GGUF_TYPE["str"]:
                out[key] = [lib.gguf_get_arr_str(g, i, j) for j in range(n)]
            else:
                dt = np.dtype(_NP[at])
                if n == 0:
                    out[key] = np.zeros(0, dt)
                else:
                    raw = (ctypes.c_uint8 * (n * dt.itemsize)).from_address(lib.gguf_get_arr_data(g, i))
                    out[key] = np.frombuffer(bytes(raw), dtype=dt)
        else:
            out[key] = getattr(lib, "gguf_get_val_" + _GETTER[t])(g, i)
    return out


def set_kv(lib: G.Lib, g, key: str, kind: str, value):
    """gguf_set_val_<kind> / gguf_set_arr_data / gguf_set_arr_str (kind 'arr:<elem>')."""
    k = key.encode()
    if kind == "str":
        lib.gguf_set_val_str(g, k, value.encode() if isinstance(value, str) else value)
    elif kind == "arr:str":
        arr = (ctypes.c_char_p * len(value))(*[v.encode() if isinstance(v, str) else v for v in value])
        lib.gguf_set_arr_str(g, k, arr, len(value))
    elif kind.startswith("arr:"):
        et = GGUF_TYPE[kind[4:]]
        a = np.ascontiguousarray(np.asarray(value, dtype=_NP[et]))
        lib.gguf_set_arr_data(g, k, et, a.ctypes.data, len(a))
    else:
        getattr(lib, "gguf_set_val_" + kind)(g, k, value)


def write(lib: G.Lib, path: str, kvs, tensors, only_meta: bool = False):
    """kvs: [(key, kind, value)]; tensors: [(name, ggml_type, ne list, raw data ndarray)]."""
    g = lib.gguf_init_empty()
    overhead = lib.ggml_tensor_overhead() * max(1, len(tensors))
    ctx = lib.ggml_init(G.ggml_init_params(overhead, None, True))
    keep = []
    try:
        for key, kind, value in kvs:
            set_kv(lib, g, key, kind, value)
        for name, t, ne, data in tensors:
            ne = list(ne) + [1] * (4 - len(ne))
            x = lib.ggml_new_tensor_4d(ctx, t, *ne)
            lib.ggml_set_name(x, name.encode())
            buf = np.ascontiguousarray(data).view(np.uint8).reshape(-1)
            assert buf.size == lib.ggml_nbytes(x), (name, buf.size, lib.ggml_nbytes(x))
            keep.append(buf)
            x.contents.data = buf.ctypes.data
            lib.gguf_add_tensor(g, x)
        lib.gguf_write_to_file(g, path.encode(), only_meta)
    finally:
        lib.ggml_free(ctx)
        lib.gguf_free(g)
