"""Q4_0 / Q8_0 decode GEMVs on the 16-byte-aligned repacked weight copies (mmq_planes.hip
k_q40_repack / k_q80_repack, mmv_fused_impl.h FmtQ0R / FmtQ8R; round 6).

The canonical block_q4_0 / block_q8_0 (ggml-common.h: f16 d + 16 / 32 quant bytes = 18 / 34 B)
leave the quants 2-byte aligned. In tree order the backend streams a per-row repacked copy instead -- all the row's quant
bytes, then all its scales -- kept next to the canonical bytes by the planes cache, which every
backend write path renews. The pair arithmetic is shared with the canonical-layout kernel, so:
  * repacked vs canonical (q40r / q80r 0): bit-identical, and both within the exact-path tolerance
    of the reference's vec_dot_q4_0_q8_0 / vec_dot_q8_0_q8_0 (ggml-quants.c:3469-3874, :4819) via
    the oracle;
  * set_tensor / get_tensor keep returning the reference bytes, and partial or asynchronous weight
    writes reach the copy (the next GEMV sees the new rows);
  * the copy is dropped with its buffer.
"""
import ctypes

import numpy as np
import pytest

import pyoracle as orc
from ggml_mi355x import ggml as G
from ggml_mi355x import synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rt():
    return G.runtime()


@pytest.fixture(scope="module")
def backend(rt):
    b = G.mi355x_backend(rt, 0)
    yield b
    rt.ggml_backend_free(b)


def rel_err(y, ref):
    return float(np.abs(y.astype(np.float64) - ref).max() / max(np.abs(ref).max(), 1e-30))


def _stats(rt):
    b = ctypes.c_size_t(0)
    return int(rt.ggml_backend_mi355x_planes_stats(ctypes.byref(b))), int(b.value)


KNOB = {"q4_0": b"q40r", "q8_0": b"q80r"}


@pytest.mark.parametrize("tname", ["q4_0", "q8_0"])
@pytest.mark.parametrize("K,N,B", [(256, 64, 1), (768, 2304, 1), (4096, 4096, 1), (4096, 300, 1), (3072, 768, 1), (11008, 130, 1),
                                   (1024, 4097, 1), (4096, 512, 2)])
def test_q40_repacked_gemv_bit_equal_canonical(rt, backend, tname, K, N, B):
    """One column on the aligned copy (several columns keep the canonical blocks: measured faster
    there for Q4_0), bit-identical to the canonical-layout kernel."""
    t = orc.TYPES_BY_NAME[tname]
    knob = KNOB[tname]
    wq = orc.quantize(t, synth.uniform(K + 7 * N, K * N), K)
    x = synth.uniform(K + 9 * B, K * B)
    n0, _ = _stats(rt)
    assert rt.ggml_backend_mi355x_set_tuning(b"mmv_order", 0)
    try:
        assert rt.ggml_backend_mi355x_set_tuning(knob, 0)
        canon = G.mul_mat_once(rt, backend, t, wq, K, N, x, B)
        assert _stats(rt)[0] == n0, "knob 0 must not create a copy"
        assert rt.ggml_backend_mi355x_set_tuning(knob, 1)
        before = _stats(rt)[0]
        rep = G.mul_mat_once(rt, backend, t, wq, K, N, x, B)
        if B > 1:
            assert _stats(rt)[0] == before
    finally:
        rt.ggml_backend_mi355x_set_tuning(knob, 1)
        rt.ggml_backend_mi355x_set_tuning(b"mmv_order", -1)
    assert _stats(rt)[0] == n0, "the copy of a freed buffer must be dropped with it"
    assert np.array_equal(rep.view(np.uint32), canon.view(np.uint32)), rel_err(rep, canon)
    assert rel_err(rep, orc.mul_mat(t, wq, K, N, x, B)) <= 1e-5


@pytest.mark.parametrize("tname", ["q4_0", "q8_0"])
def test_q40_repacked_follows_weight_writes(rt, backend, tname):
    """set_tensor at an offset (rows 37..120) and an async write (rows 150..169) renew the copy;
    get_tensor returns the canonical bytes; the copy exists while the buffer lives."""
    t = orc.TYPES_BY_NAME[tname]
    knob = KNOB[tname]
    K, N, B = 4096, 192, 1
    rb = orc.row_size(t, K)
    wq = orc.quantize(t, synth.uniform(181, K * N), K)
    wq2 = orc.quantize(t, synth.uniform(182, K * N), K)
    x = synth.uniform(183, K * B)
    ovh = rt.ggml_tensor_overhead() * 8 + rt.ggml_graph_overhead()
    assert rt.ggml_backend_mi355x_set_tuning(b"mmv_order", 0)
    try:
        with G.Context(rt, ovh, no_alloc=True) as c:
            w = rt.ggml_new_tensor_2d(c.ctx, t, K, N)
            xt = rt.ggml_new_tensor_2d(c.ctx, G.GGML_TYPE_F32, K, B)
            y = rt.ggml_mul_mat(c.ctx, w, xt)
            g = rt.ggml_new_graph(c.ctx)
            rt.ggml_build_forward_expand(g, y)
            buf = rt.ggml_backend_alloc_ctx_tensors(c.ctx, backend)
            assert buf
            try:
                n0, _ = _stats(rt)
                G.tensor_set(rt, w, wq)
                G.tensor_set(rt, xt, x)
                assert rt.ggml_backend_graph_compute(backend, g) == G.GGML_STATUS_SUCCESS
                n1, nbytes = _stats(rt)
                assert n1 == n0 + 1 and nbytes >= rb * N, "the decode GEMV did not create the aligned copy"
                assert rel_err(G.tensor_get(rt, y), orc.mul_mat(t, wq, K, N, x, B)) <= 1e-5
                back = np.empty_like(wq)
                rt.ggml_backend_tensor_get(w, back.ctypes.data, 0, back.nbytes)
                assert np.array_equal(back, wq), "get_tensor must return the canonical bytes"
                mixed = wq.copy()
                lo, hi = 37 * rb, 121 * rb
                mixed[lo:hi] = wq2[lo:hi]
                G.tensor_set(rt, w, wq2[lo:hi], offset=lo)
                assert rt.ggml_backend_graph_compute(backend, g) == G.GGML_STATUS_SUCCESS
                y2 = G.tensor_get(rt, y)
                assert rel_err(y2, orc.mul_mat(t, mixed, K, N, x, B)) <= 1e-5
                lo2, hi2 = 150 * rb, 170 * rb
                chunk = np.ascontiguousarray(wq2[lo2:hi2])
                mixed[lo2:hi2] = chunk
                rt.ggml_backend_tensor_set_async(backend, w, chunk.ctypes.data, lo2, chunk.nbytes)
                assert rt.ggml_backend_graph_compute(backend, g) == G.GGML_STATUS_SUCCESS
                rt.ggml_backend_synchronize(backend)
                y3 = G.tensor_get(rt, y)
                assert rel_err(y3, orc.mul_mat(t, mixed, K, N, x, B)) <= 1e-5
                rt.ggml_backend_tensor_get(w, back.ctypes.data, 0, back.nbytes)
                assert np.array_equal(back, mixed)
                # the canonical kernel on the same (written) bytes: the same bits
                assert rt.ggml_backend_mi355x_set_tuning(knob, 0)
                assert rt.ggml_backend_graph_compute(backend, g) == G.GGML_STATUS_SUCCESS
                y4 = G.tensor_get(rt, y)
                assert np.array_equal(y3.view(np.uint32), y4.view(np.uint32)), rel_err(y3, y4)
            finally:
                rt.ggml_backend_mi355x_set_tuning(knob, 1)
                rt.ggml_backend_buffer_free(buf)
        assert _stats(rt)[0] == n0
    finally:
        rt.ggml_backend_mi355x_set_tuning(b"mmv_order", -1)


def test_q40_grouped_decode_on_repacked_copies(rt, backend):
    """Several independent Q4_0 decode mul_mats of one graph (one grouped launch) on their aligned
    copies: each output bit-identical to the canonical-layout launch."""
    t = orc.Q4_0
    K, N, B, R = 4096, 512, 1, 6
    wqs = [orc.quantize(t, synth.uniform(300 + r, K * N), K) for r in range(R)]
    xs = [synth.uniform(400 + r, K * B) for r in range(R)]

    def run(q40r):
        ovh = rt.ggml_tensor_overhead() * (3 * R + 4) + rt.ggml_graph_overhead()
        with G.Context(rt, ovh, no_alloc=True) as c:
            ws = [rt.ggml_new_tensor_2d(c.ctx, t, K, N) for _ in range(R)]
            xts = [rt.ggml_new_tensor_2d(c.ctx, G.GGML_TYPE_F32, K, B) for _ in range(R)]
            ys = [rt.ggml_mul_mat(c.ctx, w, xt) for w, xt in zip(ws, xts)]
            g = rt.ggml_new_graph(c.ctx)
            for y in ys:
                rt.ggml_build_forward_expand(g, y)
            buf = rt.ggml_backend_alloc_ctx_tensors(c.ctx, backend)
            assert buf
            try:
                assert rt.ggml_backend_mi355x_set_tuning(b"q40r", q40r)
                for w, wq, xt, x in zip(ws, wqs, xts, xs):
                    G.tensor_set(rt, w, wq)
                    G.tensor_set(rt, xt, x)
                assert rt.ggml_backend_graph_compute(backend, g) == G.GGML_STATUS_SUCCESS
                assert rt.ggml_backend_mi355x_last_launch_count(backend) == 1
                return [G.tensor_get(rt, y) for y in ys]
            finally:
                rt.ggml_backend_mi355x_set_tuning(b"q40r", 1)
                rt.ggml_backend_buffer_free(buf)

    rep, canon = run(1), run(0)
    for r in range(R):
        assert np.array_equal(rep[r].view(np.uint32), canon[r].view(np.uint32)), (r, rel_err(rep[r], canon[r]))
    assert rel_err(rep[R - 1], orc.mul_mat(t, wqs[R - 1], K, N, xs[R - 1], B)) <= 1e-5
