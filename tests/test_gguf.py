"""GGUF files (formats): the runtime's gguf_* (csrc/core/gguf.cpp) against the
reference's own implementation (src/ggml.c:21671-22866, compiled into oracle/_ref/libggml_ref.so;
test infrastructure only).

* the same gguf_set_* / gguf_add_tensor calls write byte-identical files in both libraries;
* each library reads the other's files with identical key/values, tensor infos, data offsets and
  (no_alloc=false) tensor bytes; gguf_get_meta_size / gguf_get_meta_data agree;
* malformed files (bad magic, GGUFv1, every truncation point of the metadata) give NULL;
* on the GPU: a GGUF file's Q4_K / Q8_0 / F16 weights loaded into an MI355X buffer
  (ggml_mi355x.gguf.Model) and multiplied give the oracle's result.
"""
import ctypes
import os

import numpy as np
import pytest

from conftest import REPO

import pyoracle as orc
from ggml_mi355x import ggml as G
from ggml_mi355x import gguf
from ggml_mi355x import synth

REF_LIB = os.path.join(REPO, "oracle", "_ref", "libggml_ref.so")
needs_ref = pytest.mark.skipif(not os.path.exists(REF_LIB), reason="make -C oracle ref")

KVS = [
    ("general.name", "str", "synthetic gguf"),
    ("t.u8", "u8", 200), ("t.i8", "i8", -100), ("t.u16", "u16", 60000), ("t.i16", "i16", -30000),
    ("t.u32", "u32", 4000000000), ("t.i32", "i32", -2000000000), ("t.f32", "f32", 1.5),
    ("t.u64", "u64", 2**63 + 5), ("t.i64", "i64", -2**62), ("t.f64", "f64", 3.25), ("t.bool", "bool", True),
    ("t.arr_i32", "arr:i32", [1, -2, 3]), ("t.arr_f32", "arr:f32", [0.5, 1.5]), ("t.arr_u8_empty", "arr:u8", []),
    ("t.arr_str", "arr:str", ["a", "bc", "", "unicode é"]), ("t.str_empty", "str", ""),
]


def _tensors():
    w4 = orc.quantize(orc.Q4_K, synth.uniform(1, 256 * 3), 256)
    w0 = orc.quantize(orc.Q4_0, synth.uniform(2, 64 * 5), 64)
    w8 = orc.quantize(orc.Q8_0, synth.uniform(3, 96 * 2), 96)
    h = synth.uniform(4, 7 * 3).astype(np.float16)  # 42 bytes: exercises the padding
    f = synth.uniform(5, 5)
    i = np.arange(3, dtype=np.int32)
    return [("blk.0.q4k", orc.Q4_K, [256, 3], w4), ("blk.0.q40", orc.Q4_0, [64, 5], w0), ("q80", orc.Q8_0, [96, 2], w8),
            ("h", G.GGML_TYPE_F16, [7, 3], h), ("norm", G.GGML_TYPE_F32, [5], f), ("ids", G.GGML_TYPE_I32, [3], i),
            ("cube", G.GGML_TYPE_F32, [2, 2, 2, 2], synth.uniform(6, 16))]


@pytest.fixture(scope="module")
def libs():
    ours = G.runtime()
    ref = G.Lib([REF_LIB], isolated=True) if os.path.exists(REF_LIB) else None
    return ours, ref


def _read_all(lib, path, no_alloc):
    ctxp = ctypes.c_void_p()
    g = lib.gguf_init_from_file(path.encode(), G.gguf_init_params(no_alloc, ctypes.pointer(ctxp)))
    assert g, path
    try:
        info = {
            "version": lib.gguf_get_version(g), "alignment": lib.gguf_get_alignment(g),
            "data_offset": lib.gguf_get_data_offset(g), "kv": gguf.read_kv(lib, g),
            "tensors": [(lib.gguf_get_tensor_name(g, i), lib.gguf_get_tensor_type(g, i), lib.gguf_get_tensor_offset(g, i))
                        for i in range(lib.gguf_get_n_tensors(g))],
        }
        shapes, data = [], {}
        t = lib.ggml_get_first_tensor(ctxp.value)
        while t:
            c = t.contents
            shapes.append((c.name, c.type, tuple(c.ne)))
            if not no_alloc and c.name != b"":
                n = lib.ggml_nbytes(t)
                data[c.name] = bytes((ctypes.c_uint8 * n).from_address(c.data))
            t = lib.ggml_get_next_tensor(ctxp.value, t)
        info["ctx_tensors"] = shapes
        info["data"] = data
        return info
    finally:
        lib.ggml_free(ctxp.value)
        lib.gguf_free(g)


def _same_kv(a, b):
    assert a.keys() == b.keys()
    for k in a:
        if isinstance(a[k], np.ndarray):
            assert a[k].dtype == b[k].dtype and np.array_equal(a[k], b[k]), k
        else:
            assert a[k] == b[k], k


@needs_ref
@pytest.mark.parametrize("alignment", [None, 64])
def test_written_files_byte_identical(libs, tmp_path, alignment):
    ours, ref = libs
    kvs = KVS + ([("general.alignment", "u32", alignment)] if alignment else [])
    po, pr = str(tmp_path / "ours.gguf"), str(tmp_path / "ref.gguf")
    gguf.write(ours, po, kvs, _tensors())
    gguf.write(ref, pr, kvs, _tensors())
    a, b = open(po, "rb").read(), open(pr, "rb").read()
    assert len(a) == len(b) and a == b
    # metadata only: same bytes, and gguf_get_meta_size is their length
    gguf.write(ours, po + ".meta", kvs, _tensors(), only_meta=True)
    gguf.write(ref, pr + ".meta", kvs, _tensors(), only_meta=True)
    assert open(po + ".meta", "rb").read() == open(pr + ".meta", "rb").read()


@needs_ref
@pytest.mark.parametrize("no_alloc", [True, False])
def test_cross_read(libs, tmp_path, no_alloc):
    ours, ref = libs
    path = str(tmp_path / "m.gguf")
    for writer in (ours, ref):
        gguf.write(writer, path, KVS, _tensors())
        a, b = _read_all(ours, path, no_alloc), _read_all(ref, path, no_alloc)
        for k in ("version", "alignment", "data_offset", "tensors", "ctx_tensors"):
            assert a[k] == b[k], k
        _same_kv(a["kv"], b["kv"])
        assert a["data"].keys() == b["data"].keys()
        for name in a["data"]:
            assert a["data"][name] == b["data"][name], name
    # and the values are the ones written
    kv = a["kv"]
    assert kv["general.name"] == b"synthetic gguf" and kv["t.u64"] == 2**63 + 5 and kv["t.bool"] is True
    assert kv["t.arr_str"] == [b"a", b"bc", b"", "unicode é".encode()]
    if not no_alloc:
        for name, _, _, arr in _tensors():
            assert a["data"][name.encode()] == np.ascontiguousarray(arr).tobytes()


@needs_ref
def test_meta_size_and_data(libs):
    ours, ref = libs
    out = []
    for lib in (ours, ref):
        g = lib.gguf_init_empty()
        try:
            for k in KVS:
                gguf.set_kv(lib, g, *k)
            n = lib.gguf_get_meta_size(g)
            buf = (ctypes.c_uint8 * n)()
            lib.gguf_get_meta_data(g, buf)
            out.append(bytes(buf))
        finally:
            lib.gguf_free(g)
    assert out[0] == out[1] and len(out[0]) % 32 == 0


@needs_ref
def test_edit_operations_match(libs, tmp_path):
    """Overwrite a key with another type, remove keys, gguf_set_kv copy, retype a tensor and
    replace its data (offsets of the following tensors move): identical files."""
    ours, ref = libs
    blobs = []
    for lib in (ours, ref):
        src = lib.gguf_init_empty()
        g = lib.gguf_init_empty()
        ctx = lib.ggml_init(G.ggml_init_params(lib.ggml_tensor_overhead() * 8, None, True))
        keep = []
        try:
            for k in KVS:
                gguf.set_kv(lib, src, *k)
            lib.gguf_set_kv(g, src)
            gguf.set_kv(lib, g, "t.u8", "str", "now a string")
            gguf.set_kv(lib, g, "general.name", "arr:i16", [7, 8])
            lib.gguf_remove_key(g, b"t.f32")
            lib.gguf_remove_key(g, b"no.such.key")
            for name, t, ne, arr in _tensors():
                x = lib.ggml_new_tensor_4d(ctx, t, *(list(ne) + [1] * (4 - len(ne))))
                lib.ggml_set_name(x, name.encode())
                b = np.ascontiguousarray(arr).view(np.uint8).reshape(-1)
                keep.append(b)
                x.contents.data = b.ctypes.data
                lib.gguf_add_tensor(g, x)
            repl = np.arange(100, dtype=np.uint8)
            keep.append(repl)
            lib.gguf_set_tensor_type(g, b"h", 24)  # GGML_TYPE_I8
            lib.gguf_set_tensor_data(g, b"h", repl.ctypes.data, 100)
            assert lib.gguf_find_key(g, b"t.f32") == -1 and lib.gguf_find_tensor(g, b"cube") == 6
            p = str(tmp_path / f"edit{len(blobs)}.gguf")
            lib.gguf_write_to_file(g, p.encode(), False)
            blobs.append(open(p, "rb").read())
        finally:
            lib.ggml_free(ctx)
            lib.gguf_free(g)
            lib.gguf_free(src)
    assert blobs[0] == blobs[1]


def test_malformed_files_return_null(libs, tmp_path):
    ours, ref = libs
    path = str(tmp_path / "ok.gguf")
    gguf.write(ours, path, KVS, _tensors())
    good = open(path, "rb").read()
    bad = str(tmp_path / "bad.gguf")
    cases = [b"GGUX" + good[4:], good[:4] + (1).to_bytes(4, "little") + good[8:]]
    g = ours.gguf_init_from_file(path.encode(), G.gguf_init_params(True, None))
    meta_end = ours.gguf_get_data_offset(g)
    ours.gguf_free(g)
    cases += [good[:n] for n in sorted(set(list(range(0, 64, 3)) + list(range(64, meta_end, 37))))]
    for blob in cases:
        open(bad, "wb").write(blob)
        for lib in (ours,) + ((ref,) if ref else ()):
            ctxp = ctypes.c_void_p()
            assert not lib.gguf_init_from_file(bad.encode(), G.gguf_init_params(False, ctypes.pointer(ctxp))), len(blob)
    assert not ours.gguf_init_from_file(str(tmp_path / "missing.gguf").encode(), G.gguf_init_params(True, None))


@pytest.mark.gpu
def test_gguf_weights_on_mi355x_mul_mat(libs, tmp_path):
    """GGUF -> MI355X buffer (gguf.Model) -> MUL_MAT on the device: the oracle's result."""
    ours, _ = libs
    K, N, B = 1024, 96, 3
    ws = {t: synth.uniform(10 + t, K * N) for t in (orc.Q4_K, orc.Q8_0)}
    tens = [(f"w{t}", t, [K, N], orc.quantize(t, ws[t], K)) for t in ws]
    tens.append(("wh", G.GGML_TYPE_F16, [K, N], synth.uniform(9, K * N).astype(np.float16)))
    path = str(tmp_path / "w.gguf")
    gguf.write(ours, path, [("general.architecture", "str", "test")], tens)
    be = G.mi355x_backend(ours)
    m = gguf.Model(ours, path, be)
    try:
        assert m.kv["general.architecture"] == b"test"
        x = synth.uniform(77, K * B)
        for name, t, _, wq in tens:
            w = m.tensors[name]
            back = np.empty(ours.ggml_nbytes(w), np.uint8)
            ours.ggml_backend_tensor_get(w, back.ctypes.data, 0, back.nbytes)
            assert np.array_equal(back, np.ascontiguousarray(wq).view(np.uint8).reshape(-1))

            def build(c, w=w):
                xt = ours.ggml_new_tensor_2d(c, G.GGML_TYPE_F32, K, B)
                return [(xt, x)], ours.ggml_mul_mat(c, w, xt)

            y = G.graph_once(ours, be, build)
            yr = orc.mul_mat(t, np.ascontiguousarray(wq).view(np.uint8).reshape(-1), K, N, x, B)
            err = float(np.abs(y - yr).max() / np.abs(yr).max())
            assert err <= 1e-3, (name, err)
    finally:
        m.free()
        ours.ggml_backend_free(be)
