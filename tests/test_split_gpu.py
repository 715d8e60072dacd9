"""GPU tests of the tensor-split row path (ggml_backend_mi355x_split_buffer_type, analogue of
ggml_backend_cuda_split_buffer_type, src/ggml-cuda.cu:578-975 / :1360-1647).

The weight's rows are divided over 3 slots. On a one-GPU box GGML_MI355X_SPLIT_SLOTS=3 puts slots
1 and 2 on device 0 as well, each with its own allocation, stream and copies, so the multi-device
path (src1 copied in, per-slot GEMM on the slot's stream, row slices gathered into dst under
events) is what runs; on a multi-GPU node the same code peer-copies over xGMI. The split result is
checked against the oracle within the north_star tolerance and against the unsplit backend result
(which may take the grouped decode kernel, whose f32 combination order differs) within 1e-5.
"""
import ctypes
import os

os.environ.setdefault("GGML_MI355X_SPLIT_SLOTS", "3")  # read once, at the first split buffer type

import numpy as np
import pytest

import pyoracle as orc
from ggml_mi355x import ggml as G
from ggml_mi355x import synth

pytestmark = pytest.mark.gpu

TOL = 1e-3


@pytest.fixture(scope="module")
def rt():
    return G.runtime()


@pytest.fixture(scope="module")
def backend(rt):
    b = G.mi355x_backend(rt, 0)
    yield b
    rt.ggml_backend_free(b)


def rel(y, ref):
    return float(np.abs(y.astype(np.float64) - ref).max() / max(np.abs(ref).max(), 1e-30))


def split_buft(rt, props):
    if props is None:
        return rt.ggml_backend_mi355x_split_buffer_type(None)
    arr = (ctypes.c_float * 16)(*([float(p) for p in props] + [0.0] * (16 - len(props))))
    return rt.ggml_backend_mi355x_split_buffer_type(ctypes.cast(arr, ctypes.c_void_p))


def mul_mat_split(rt, backend, buft, t, wq, K, N, x, B, extra_add=False):
    """W (in the split buffer type) x X -> Y; optionally Y + Y as a following node."""
    cw = G.Context(rt, rt.ggml_tensor_overhead() * 4, no_alloc=True)
    cx = G.Context(rt, rt.ggml_tensor_overhead() * 8 + rt.ggml_graph_overhead(), no_alloc=True)
    try:
        w = rt.ggml_new_tensor_2d(cw.ctx, t, K, N)
        wbuf = rt.ggml_backend_alloc_ctx_tensors_from_buft(cw.ctx, buft)
        assert wbuf
        assert rt.ggml_backend_buffer_name(wbuf) == b"MI355X_Split"
        assert not rt.ggml_backend_buffer_is_host(wbuf)
        assert rt.ggml_backend_buft_get_alloc_size(buft, w) >= rt.ggml_nbytes(w)
        xt = rt.ggml_new_tensor_2d(cx.ctx, G.GGML_TYPE_F32, K, B)
        y = rt.ggml_mul_mat(cx.ctx, w, xt)
        out = rt.ggml_add(cx.ctx, y, y) if extra_add else y
        g = rt.ggml_new_graph(cx.ctx)
        rt.ggml_build_forward_expand(g, out)
        xbuf = rt.ggml_backend_alloc_ctx_tensors(cx.ctx, backend)
        try:
            G.tensor_set(rt, w, wq)
            back = np.empty_like(wq)
            rt.ggml_backend_tensor_get(w, back.ctypes.data, 0, back.nbytes)
            assert np.array_equal(back, wq), "split set/get round trip"
            G.tensor_set(rt, xt, x.astype(np.float32))
            assert rt.ggml_backend_graph_compute(backend, g) == G.GGML_STATUS_SUCCESS
            return G.tensor_get(rt, out)
        finally:
            rt.ggml_backend_buffer_free(xbuf)
            rt.ggml_backend_buffer_free(wbuf)
    finally:
        cx.free()
        cw.free()


@pytest.mark.parametrize("tname", ["q4_K", "q5_K", "q4_0", "q8_0", "f16", "f32"])
@pytest.mark.parametrize("B", [1, 5, 64])
def test_split_mul_mat_matches_unsplit(rt, backend, tname, B):
    t = orc.TYPES_BY_NAME[tname]
    K, N = 2048, 1000  # 1000 rows over [1, 2, 1]: slices 0-191, 192-703, 704-999 (64-row rounding)
    w = synth.uniform(7 + B, K * N)
    x = synth.uniform(11 + B, K * B)
    wq = orc.quantize(t, w, K)
    y_split = mul_mat_split(rt, backend, split_buft(rt, [1, 2, 1]), t, wq, K, N, x, B)
    y_ref = G.mul_mat_once(rt, backend, t, wq, K, N, x, B)
    assert rel(y_split, y_ref) <= 1e-5
    assert rel(y_split, orc.mul_mat(t, wq, K, N, x, B)) <= TOL


def test_split_default_and_uneven(rt, backend):
    t = orc.Q4_K
    K, N, B = 1024, 777, 3
    w = synth.uniform(3, K * N)
    x = synth.uniform(4, K * B)
    wq = orc.quantize(t, w, K)
    y_ref = G.mul_mat_once(rt, backend, t, wq, K, N, x, B)
    for props in (None, [0, 1, 0], [5, 0, 1]):  # equal split; everything on one slot; an empty slot
        y = mul_mat_split(rt, backend, split_buft(rt, props), t, wq, K, N, x, B, extra_add=True)
        assert rel(y, y_ref + y_ref) <= 1e-5, props


def test_split_buffer_type_is_cached(rt):
    assert split_buft(rt, [1, 2, 1]) == split_buft(rt, [2, 4, 2])  # same normalised split
    assert split_buft(rt, [1, 2, 1]) != split_buft(rt, [1, 1, 1])
