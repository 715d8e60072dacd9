"""ctypes mirror of the ggml C API (include/ggml_abi.h) -- host-side harness of the runtime.

The same wrapper binds either library exporting the reference API:
  * the MI355X runtime: lib/libggml_core.so (+ the backend lib/libggml_mi355x.so), or
  * the reference libggml (oracle/_ref/libggml_ref.so, tests only),
so a test can build the identical graph on both and compare, the way the reference's own
test-backend-ops compares a backend against the CPU (tests/test-backend-ops.cpp:358-515).
"""
from __future__ import annotations

import ctypes
import os
from ctypes import (POINTER, Structure, c_bool, c_char, c_char_p, c_float, c_int, c_int32, c_int64, c_size_t,
                    c_uint8, c_void_p)

import numpy as np

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_DIR = os.path.join(PKG_ROOT, "lib")
# GGML_MI355X_CORE_LIB: an alternative build of the host runtime (the sanitizer build of
# `make -C ggml-imax_amd sanitize`, run by tools/sanitize.sh)
CORE_LIB = os.environ.get("GGML_MI355X_CORE_LIB") or os.path.join(LIB_DIR, "libggml_core.so")
# GGML_MI355X_BACKEND_LIB: an alternative build of the backend (A/B builds, e.g. `make abpk`)
BACKEND_LIB = os.environ.get("GGML_MI355X_BACKEND_LIB") or os.path.join(LIB_DIR, "libggml_mi355x.so")
GPT2_LIB = os.path.join(LIB_DIR, "libgpt2_mi355x.so")

# enum ggml_type (include/ggml/ggml.h:348-381)
GGML_TYPE_F32, GGML_TYPE_F16, GGML_TYPE_Q4_0, GGML_TYPE_Q8_0 = 0, 1, 2, 8
GGML_TYPE_Q4_K, GGML_TYPE_Q5_K, GGML_TYPE_Q8_K, GGML_TYPE_I32 = 12, 13, 15, 26
TYPE_BY_NAME = {"f32": 0, "f16": 1, "q4_0": 2, "q8_0": 8, "q4_K": 12, "q5_K": 13, "i32": 26}
BLOCK = {0: (1, 4), 1: (1, 2), 2: (32, 18), 8: (32, 34), 12: (256, 144), 13: (256, 176), 26: (1, 4)}

GGML_OP_MUL_MAT = 23
GGML_STATUS_SUCCESS = 0


def row_size(t: int, n: int) -> int:
    blk, sz = BLOCK[t]
    assert n % blk == 0
    return n // blk * sz


class ggml_tensor(Structure):
    _fields_ = [
        ("type", c_int), ("backend", c_int), ("buffer", c_void_p),
        ("ne", c_int64 * 4), ("nb", c_size_t * 4),
        ("op", c_int), ("op_params", c_int32 * 16), ("flags", c_int32),
        ("grad", c_void_p), ("src", c_void_p * 10),
        ("perf_runs", c_int), ("perf_cycles", c_int64), ("perf_time_us", c_int64),
        ("view_src", c_void_p), ("view_offs", c_size_t), ("data", c_void_p),
        ("name", c_char * 64), ("extra", c_void_p), ("padding", c_char * 8),
    ]


assert ctypes.sizeof(ggml_tensor) == 368, ctypes.sizeof(ggml_tensor)


class ggml_init_params(Structure):
    _fields_ = [("mem_size", c_size_t), ("mem_buffer", c_void_p), ("no_alloc", c_bool)]


class gguf_init_params(Structure):
    _fields_ = [("no_alloc", c_bool), ("ctx", POINTER(c_void_p))]


class ggml_cgraph(Structure):
    _fields_ = [("size", c_int), ("n_nodes", c_int), ("n_leafs", c_int),
                ("nodes", POINTER(POINTER(ggml_tensor))), ("grads", c_void_p), ("leafs", POINTER(POINTER(ggml_tensor))),
                ("hash_size", c_size_t), ("hash_keys", c_void_p), ("order", c_int),
                ("perf_runs", c_int), ("perf_cycles", c_int64), ("perf_time_us", c_int64)]


T = POINTER(ggml_tensor)

_SIGS = {
    # core
    "ggml_init": ([ggml_init_params], c_void_p),
    "ggml_free": ([c_void_p], None),
    "ggml_tensor_overhead": ([], c_size_t),
    "ggml_graph_overhead": ([], c_size_t),
    "ggml_graph_overhead_custom": ([c_size_t, c_bool], c_size_t),
    "ggml_new_tensor_1d": ([c_void_p, c_int, c_int64], T),
    "ggml_new_tensor_2d": ([c_void_p, c_int, c_int64, c_int64], T),
    "ggml_new_tensor_3d": ([c_void_p, c_int, c_int64, c_int64, c_int64], T),
    "ggml_new_tensor_4d": ([c_void_p, c_int, c_int64, c_int64, c_int64, c_int64], T),
    "ggml_set_name": ([T, c_char_p], T),
    "ggml_nbytes": ([T], c_size_t),
    "ggml_nelements": ([T], c_int64),
    "ggml_type_size": ([c_int], c_size_t),
    "ggml_blck_size": ([c_int], c_int),
    "ggml_row_size": ([c_int, c_int64], c_size_t),
    "ggml_type_name": ([c_int], c_char_p),
    "ggml_op_name": ([c_int], c_char_p),
    "ggml_op_desc": ([T], c_char_p),
    "ggml_is_contiguous": ([T], c_bool),
    "ggml_mul_mat": ([c_void_p, T, T], T),
    "ggml_add": ([c_void_p, T, T], T),
    "ggml_mul": ([c_void_p, T, T], T),
    "ggml_scale": ([c_void_p, T, c_float], T),
    "ggml_norm": ([c_void_p, T, c_float], T),
    "ggml_rms_norm": ([c_void_p, T, c_float], T),
    "ggml_gelu": ([c_void_p, T], T),
    "ggml_silu": ([c_void_p, T], T),
    "ggml_soft_max": ([c_void_p, T], T),
    "ggml_soft_max_ext": ([c_void_p, T, T, c_float, c_float], T),
    "ggml_diag_mask_inf": ([c_void_p, T, c_int], T),
    "ggml_get_rows": ([c_void_p, T, T], T),
    "ggml_rope": ([c_void_p, T, T, c_int, c_int, c_int], T),
    "ggml_cpy": ([c_void_p, T, T], T),
    "ggml_cont": ([c_void_p, T], T),
    "ggml_transpose": ([c_void_p, T], T),
    "ggml_permute": ([c_void_p, T, c_int, c_int, c_int, c_int], T),
    "ggml_view_1d": ([c_void_p, T, c_int64, c_size_t], T),
    "ggml_view_2d": ([c_void_p, T, c_int64, c_int64, c_size_t, c_size_t], T),
    "ggml_cont_2d": ([c_void_p, T, c_int64, c_int64], T),
    "ggml_cont_3d": ([c_void_p, T, c_int64, c_int64, c_int64], T),
    "ggml_view_3d": ([c_void_p, T, c_int64, c_int64, c_int64, c_size_t, c_size_t, c_size_t], T),
    "ggml_reshape_3d": ([c_void_p, T, c_int64, c_int64, c_int64], T),
    "ggml_new_graph": ([c_void_p], POINTER(ggml_cgraph)),
    "ggml_new_graph_custom": ([c_void_p, c_size_t, c_bool], POINTER(ggml_cgraph)),
    "ggml_build_forward_expand": ([POINTER(ggml_cgraph), T], None),
    "ggml_graph_print": ([POINTER(ggml_cgraph)], None),
    "ggml_quantize_chunk": ([c_int, c_void_p, c_void_p, c_int64, c_int64, c_int64, c_void_p], c_size_t),
    "ggml_fp32_to_fp16": ([c_float], ctypes.c_uint16),
    "ggml_fp16_to_fp32": ([ctypes.c_uint16], c_float),
    # GGUF (include/ggml/ggml.h:2247-2380)
    "gguf_init_empty": ([], c_void_p),
    "gguf_init_from_file": ([c_char_p, gguf_init_params], c_void_p),
    "gguf_free": ([c_void_p], None),
    "gguf_type_name": ([c_int], c_char_p),
    "gguf_get_version": ([c_void_p], c_int),
    "gguf_get_alignment": ([c_void_p], c_size_t),
    "gguf_get_data_offset": ([c_void_p], c_size_t),
    "gguf_get_data": ([c_void_p], c_void_p),
    "gguf_get_n_kv": ([c_void_p], c_int),
    "gguf_find_key": ([c_void_p, c_char_p], c_int),
    "gguf_get_key": ([c_void_p, c_int], c_char_p),
    "gguf_get_kv_type": ([c_void_p, c_int], c_int),
    "gguf_get_arr_type": ([c_void_p, c_int], c_int),
    "gguf_get_val_u8": ([c_void_p, c_int], ctypes.c_uint8),
    "gguf_get_val_i8": ([c_void_p, c_int], ctypes.c_int8),
    "gguf_get_val_u16": ([c_void_p, c_int], ctypes.c_uint16),
    "gguf_get_val_i16": ([c_void_p, c_int], ctypes.c_int16),
    "gguf_get_val_u32": ([c_void_p, c_int], ctypes.c_uint32),
    "gguf_get_val_i32": ([c_void_p, c_int], ctypes.c_int32),
    "gguf_get_val_f32": ([c_void_p, c_int], c_float),
    "gguf_get_val_u64": ([c_void_p, c_int], ctypes.c_uint64),
    "gguf_get_val_i64": ([c_void_p, c_int], c_int64),
    "gguf_get_val_f64": ([c_void_p, c_int], ctypes.c_double),
    "gguf_get_val_bool": ([c_void_p, c_int], c_bool),
    "gguf_get_val_str": ([c_void_p, c_int], c_char_p),
    "gguf_get_val_data": ([c_void_p, c_int], c_void_p),
    "gguf_get_arr_n": ([c_void_p, c_int], c_int),
    "gguf_get_arr_data": ([c_void_p, c_int], c_void_p),
    "gguf_get_arr_str": ([c_void_p, c_int, c_int], c_char_p),
    "gguf_get_n_tensors": ([c_void_p], c_int),
    "gguf_find_tensor": ([c_void_p, c_char_p], c_int),
    "gguf_get_tensor_offset": ([c_void_p, c_int], c_size_t),
    "gguf_get_tensor_name": ([c_void_p, c_int], c_char_p),
    "gguf_get_tensor_type": ([c_void_p, c_int], c_int),
    "gguf_remove_key": ([c_void_p, c_char_p], None),
    "gguf_set_val_u8": ([c_void_p, c_char_p, ctypes.c_uint8], None),
    "gguf_set_val_i8": ([c_void_p, c_char_p, ctypes.c_int8], None),
    "gguf_set_val_u16": ([c_void_p, c_char_p, ctypes.c_uint16], None),
    "gguf_set_val_i16": ([c_void_p, c_char_p, ctypes.c_int16], None),
    "gguf_set_val_u32": ([c_void_p, c_char_p, ctypes.c_uint32], None),
    "gguf_set_val_i32": ([c_void_p, c_char_p, ctypes.c_int32], None),
    "gguf_set_val_f32": ([c_void_p, c_char_p, c_float], None),
    "gguf_set_val_u64": ([c_void_p, c_char_p, ctypes.c_uint64], None),
    "gguf_set_val_i64": ([c_void_p, c_char_p, c_int64], None),
    "gguf_set_val_f64": ([c_void_p, c_char_p, ctypes.c_double], None),
    "gguf_set_val_bool": ([c_void_p, c_char_p, c_bool], None),
    "gguf_set_val_str": ([c_void_p, c_char_p, c_char_p], None),
    "gguf_set_arr_data": ([c_void_p, c_char_p, c_int, c_void_p, c_int], None),
    "gguf_set_arr_str": ([c_void_p, c_char_p, POINTER(c_char_p), c_int], None),
    "gguf_set_kv": ([c_void_p, c_void_p], None),
    "gguf_add_tensor": ([c_void_p, T], None),
    "gguf_set_tensor_type": ([c_void_p, c_char_p, c_int], None),
    "gguf_set_tensor_data": ([c_void_p, c_char_p, c_void_p, c_size_t], None),
    "gguf_write_to_file": ([c_void_p, c_char_p, c_bool], None),
    "gguf_get_meta_size": ([c_void_p], c_size_t),
    "gguf_get_meta_data": ([c_void_p, c_void_p], None),
    "ggml_get_first_tensor": ([c_void_p], T),
    "ggml_get_next_tensor": ([c_void_p, T], T),
    "ggml_get_tensor": ([c_void_p, c_char_p], T),
    # backend
    "ggml_backend_name": ([c_void_p], c_char_p),
    "ggml_backend_free": ([c_void_p], None),
    "ggml_backend_get_default_buffer_type": ([c_void_p], c_void_p),
    "ggml_backend_get_alignment": ([c_void_p], c_size_t),
    "ggml_backend_alloc_ctx_tensors": ([c_void_p, c_void_p], c_void_p),
    "ggml_backend_alloc_ctx_tensors_from_buft": ([c_void_p, c_void_p], c_void_p),
    "ggml_backend_buffer_free": ([c_void_p], None),
    "ggml_backend_buffer_get_size": ([c_void_p], c_size_t),
    "ggml_backend_buffer_get_base": ([c_void_p], c_void_p),
    "ggml_backend_buffer_name": ([c_void_p], c_char_p),
    "ggml_backend_buffer_clear": ([c_void_p, c_uint8], None),
    "ggml_backend_buffer_is_host": ([c_void_p], c_bool),
    "ggml_backend_buft_name": ([c_void_p], c_char_p),
    "ggml_backend_buft_alloc_buffer": ([c_void_p, c_size_t], c_void_p),
    "ggml_backend_buft_get_alignment": ([c_void_p], c_size_t),
    "ggml_backend_buft_get_alloc_size": ([c_void_p, T], c_size_t),
    "ggml_backend_buft_supports_backend": ([c_void_p, c_void_p], c_bool),
    "ggml_backend_tensor_set": ([T, c_void_p, c_size_t, c_size_t], None),
    "ggml_backend_tensor_get": ([T, c_void_p, c_size_t, c_size_t], None),
    "ggml_backend_tensor_set_async": ([c_void_p, T, c_void_p, c_size_t, c_size_t], None),
    "ggml_backend_graph_compute": ([c_void_p, POINTER(ggml_cgraph)], c_int),
    "ggml_backend_graph_compute_async": ([c_void_p, POINTER(ggml_cgraph)], c_int),
    "ggml_backend_synchronize": ([c_void_p], None),
    "ggml_backend_graph_plan_create": ([c_void_p, POINTER(ggml_cgraph)], c_void_p),
    "ggml_backend_graph_plan_free": ([c_void_p, c_void_p], None),
    "ggml_backend_graph_plan_compute": ([c_void_p, c_void_p], c_int),
    "ggml_backend_supports_op": ([c_void_p, T], c_bool),
    "ggml_backend_reg_get_count": ([], c_size_t),
    "ggml_backend_reg_get_name": ([c_size_t], c_char_p),
    "ggml_backend_reg_find_by_name": ([c_char_p], c_size_t),
    "ggml_backend_reg_init_backend": ([c_size_t, c_char_p], c_void_p),
    "ggml_backend_cpu_buffer_type": ([], c_void_p),
    "ggml_gallocr_new": ([c_void_p], c_void_p),
    "ggml_gallocr_free": ([c_void_p], None),
    "ggml_gallocr_reserve": ([c_void_p, POINTER(ggml_cgraph)], c_bool),
    "ggml_gallocr_alloc_graph": ([c_void_p, POINTER(ggml_cgraph)], c_bool),
    "ggml_gallocr_get_buffer_size": ([c_void_p, c_int], c_size_t),
    "ggml_tallocr_new": (None, None),  # struct by value: bound manually below
    # reference-only (CPU backend) -- absent from the MI355X runtime
    "ggml_backend_cpu_init": ([], c_void_p),
    "ggml_backend_cpu_set_n_threads": ([c_void_p, c_int], None),
    # MI355X backend
    "ggml_backend_mi355x_init": ([c_int], c_void_p),
    "ggml_backend_is_mi355x": ([c_void_p], c_bool),
    "ggml_backend_mi355x_buffer_type": ([c_int], c_void_p),
    "ggml_backend_mi355x_host_buffer_type": ([], c_void_p),
    "ggml_backend_mi355x_split_buffer_type": ([c_void_p], c_void_p),
    "ggml_backend_mi355x_get_device_count": ([], c_int),
    "ggml_backend_mi355x_get_device_description": ([c_int, c_char_p, c_size_t], None),
    "ggml_backend_mi355x_get_device_memory": ([c_int, POINTER(c_size_t), POINTER(c_size_t)], None),
    "ggml_backend_mi355x_reg_devices": ([], c_int),
    "ggml_backend_mi355x_get_stream": ([c_void_p], c_void_p),
    "ggml_backend_mi355x_last_launch_count": ([c_void_p], c_int),
    "ggml_backend_mi355x_set_tuning": ([c_char_p, c_int], c_bool),
    "ggml_backend_mi355x_set_graph_capture": ([c_void_p, c_bool], None),
    "ggml_backend_mi355x_set_perf": ([c_void_p, c_bool], None),
    "ggml_backend_mi355x_graph_stats": ([c_void_p, c_void_p], None),
    "ggml_backend_mi355x_graph_stats_ex": ([c_void_p, c_void_p, c_int], c_int),
    "ggml_backend_mi355x_stamps_enable": ([c_size_t], c_bool),
    "ggml_backend_mi355x_stamps_reset": ([], None),
    "ggml_backend_mi355x_stamps_read": ([c_void_p, c_size_t, c_char_p, c_size_t], c_size_t),
    "ggml_backend_mi355x_planes_stats": ([c_void_p], c_size_t),
    "ggml_backend_mi355x_quantize_activations": ([c_void_p, c_int, c_void_p, c_int64, c_int64, c_void_p, c_void_p, c_void_p], c_bool),
    # GPT-2 driver (include/gpt2-mi355x.h)
    "gpt2_model_load": ([c_char_p, c_void_p, c_int, c_int], c_void_p),
    "gpt2_model_load_ex": ([c_char_p, c_void_p, c_int, c_int, c_void_p], c_void_p),
    "gpt2_logits_host": ([c_void_p], c_void_p),
    "gpt2_model_free": ([c_void_p], None),
    "gpt2_model_load_sched": ([c_char_p, c_void_p, c_int, c_int, c_int, c_int], c_void_p),
    "gpt2_model_load_sched_ex": ([c_char_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p], c_void_p),
    "gpt2_sched_n_splits": ([c_void_p], c_int),
    "gpt2_model_hparams": ([c_void_p, c_void_p], None),
    "gpt2_model_size": ([c_void_p], c_size_t),
    "gpt2_compute_buffer_size": ([c_void_p], c_size_t),
    "gpt2_eval": ([c_void_p, c_int, c_void_p, c_int, c_void_p, c_int], c_int),
    "gpt2_token_text": ([c_void_p, c_int32], c_char_p),
    "gpt2_tokenize": ([c_void_p, c_char_p, c_void_p, c_int], c_int),
    "gpt2_last_eval_stats": ([c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p], None),
    "gpt2_last_eval_timing": ([c_void_p, c_void_p], None),
    "gpt2_decode_batch": ([c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int], c_int),
    "gpt2_kv_cache_seq_cp": ([c_void_p, c_int32, c_int32, c_int32, c_int32], None),
    "gpt2_kv_cache_clear": ([c_void_p], None),
    "gpt2_batch_stats": ([c_void_p, c_void_p], None),
}

BACKEND_EXPORTS = [k for k in _SIGS if k.startswith("ggml_backend_mi355x") or k == "ggml_backend_is_mi355x"]


class Lib:
    """Binds the ggml API from one or more shared libraries (first match wins)."""

    _namespaces = {}  # isolated library sets loaded by dlmopen, one link namespace each

    def __init__(self, paths, isolated: bool = False):
        # isolated: bind the library's internal calls to itself (RTLD_DEEPBIND, not global), so
        # the reference libggml and the runtime can live in one process without interposing.
        # Under AddressSanitizer (which refuses RTLD_DEEPBIND; tools/sanitize.sh sets
        # GGML_MI355X_ISOLATE=dlmopen) the set goes into a link namespace of its own instead.
        if isolated and os.environ.get("GGML_MI355X_ISOLATE") == "dlmopen":
            self.handles = Lib._dlmopen(tuple(paths))
        else:
            mode = (ctypes.RTLD_LOCAL | os.RTLD_DEEPBIND) if isolated else ctypes.RTLD_GLOBAL
            self.handles = [ctypes.CDLL(p, mode=mode) for p in paths]
        self.paths = list(paths)
        for name, (argtypes, restype) in _SIGS.items():
            if argtypes is None:
                continue
            fn = None
            for h in self.handles:
                try:
                    fn = getattr(h, name)
                    break
                except AttributeError:
                    continue
            if fn is None:
                continue
            fn.argtypes = argtypes
            fn.restype = restype
            setattr(self, name, fn)

    @staticmethod
    def _dlmopen(paths):
        if paths in Lib._namespaces:
            return Lib._namespaces[paths]
        libc = ctypes.CDLL(None)
        libc.dlmopen.restype = c_void_p
        libc.dlmopen.argtypes = [ctypes.c_long, c_char_p, c_int]
        libc.dlinfo.argtypes = [c_void_p, c_int, c_void_p]
        lmid, handles = -1, []  # LM_ID_NEWLM, then the namespace of the first library
        for p in paths:
            h = libc.dlmopen(lmid, p.encode(), 2)  # RTLD_NOW
            if not h:
                raise OSError(f"dlmopen {p} failed")
            if lmid == -1:
                lm = ctypes.c_long()
                libc.dlinfo(h, 1, ctypes.byref(lm))  # RTLD_DI_LMID
                lmid = lm.value
            handles.append(ctypes.CDLL(p, handle=h))
        Lib._namespaces[paths] = handles
        return handles

    def has(self, name: str) -> bool:
        return hasattr(self, name)


_runtime = None


def runtime() -> Lib:
    """The MI355X runtime (core + backend). Fails loudly if it has not been built."""
    global _runtime
    if _runtime is None:
        for p in (CORE_LIB, BACKEND_LIB, GPT2_LIB):
            if not os.path.exists(p):
                raise RuntimeError(f"{p} missing: run `make -C ggml-imax_amd` (or __graft_entry__.build())")
        _runtime = Lib([CORE_LIB, BACKEND_LIB, GPT2_LIB])
    return _runtime


# ------------------------------------------------------------------------------------------
# small conveniences shared by tests / bench (same calls a C program makes)
# ------------------------------------------------------------------------------------------

class Context:
    def __init__(self, lib: Lib, mem_size: int, no_alloc: bool = True):
        self.lib = lib
        self.ctx = lib.ggml_init(ggml_init_params(mem_size, None, no_alloc))
        assert self.ctx, "ggml_init failed"

    def free(self):
        if self.ctx:
            self.lib.ggml_free(self.ctx)
            self.ctx = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.free()


def tensor_set(lib: Lib, t, arr: np.ndarray, offset: int = 0):
    arr = np.ascontiguousarray(arr)
    lib.ggml_backend_tensor_set(t, arr.ctypes.data, offset, arr.nbytes)


def tensor_data_ptr(lib: Lib, t) -> int:
    """Device (or host) address of tensor t's data (ggml_tensor.data, offset 280)."""
    return int(t.contents.data or 0)


def tensor_get(lib: Lib, t, dtype=np.float32, count=None) -> np.ndarray:
    n = lib.ggml_nbytes(t)
    out = np.empty(n // np.dtype(dtype).itemsize, dtype=dtype)
    lib.ggml_backend_tensor_get(t, out.ctypes.data, 0, n)
    return out if count is None else out[:count]


def mi355x_backend(lib: Lib, device: int = 0):
    b = lib.ggml_backend_mi355x_init(device)
    if not b:
        raise RuntimeError(f"ggml_backend_mi355x_init({device}) failed (no MI355X visible?)")
    return b


def mul_mat_once(lib: Lib, backend, wtype: int, wq: np.ndarray, K: int, N: int, x: np.ndarray, B: int) -> np.ndarray:
    """Build W[K,N] (wtype) x X[K,B] f32 -> Y[N,B] on `backend`, through the public API."""
    overhead = lib.ggml_tensor_overhead() * 8 + lib.ggml_graph_overhead()
    with Context(lib, overhead, no_alloc=True) as c:
        w = lib.ggml_new_tensor_2d(c.ctx, wtype, K, N)
        xt = lib.ggml_new_tensor_2d(c.ctx, GGML_TYPE_F32, K, B)
        y = lib.ggml_mul_mat(c.ctx, w, xt)
        g = lib.ggml_new_graph(c.ctx)
        lib.ggml_build_forward_expand(g, y)
        buf = lib.ggml_backend_alloc_ctx_tensors(c.ctx, backend)
        assert buf, "buffer allocation failed"
        try:
            tensor_set(lib, w, wq)
            tensor_set(lib, xt, x.astype(np.float32))
            st = lib.ggml_backend_graph_compute(backend, g)
            assert st == GGML_STATUS_SUCCESS, st
            return tensor_get(lib, y)
        finally:
            lib.ggml_backend_buffer_free(buf)


def graph_once(lib: Lib, backend, build, n_tensors: int = 64):
    """Build a graph with `build(ctx) -> (feeds, out)` (feeds: list of (tensor, ndarray)), allocate
    it on `backend`, upload the feeds, compute, and return `out` as a float32/raw array."""
    overhead = lib.ggml_tensor_overhead() * n_tensors + lib.ggml_graph_overhead()
    with Context(lib, overhead, no_alloc=True) as c:
        feeds, out = build(c.ctx)
        g = lib.ggml_new_graph(c.ctx)
        lib.ggml_build_forward_expand(g, out)
        buf = lib.ggml_backend_alloc_ctx_tensors(c.ctx, backend)
        assert buf, "buffer allocation failed"
        try:
            for t, arr in feeds:
                tensor_set(lib, t, arr)
            st = lib.ggml_backend_graph_compute(backend, g)
            assert st == GGML_STATUS_SUCCESS, st
            o = out.contents
            return tensor_get(lib, out, np.float16 if o.type == GGML_TYPE_F16 else np.float32)
        finally:
            lib.ggml_backend_buffer_free(buf)
