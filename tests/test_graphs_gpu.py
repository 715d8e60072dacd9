"""hipGraph capture inside graph_compute (the reference CUDA backend's CUDA graphs,
src/ggml-cuda.cu:2456-2713: capture at :2576, exec update at :2690, GGML_CUDA_DISABLE_GRAPHS at
:2462) and graph plans.

A graph computed again with the same content is replayed from its capture; a graph of the same
topology with other kernel arguments updates the executable graph in place. Every replayed /
updated result must be bit-identical to the same graph launched directly (capture disabled).
"""
import ctypes

import numpy as np
import pytest

from ggml_mi355x import ggml as G
from ggml_mi355x import synth

pytestmark = pytest.mark.gpu

F32 = G.GGML_TYPE_F32


def _stats(rt, be):
    arr = (ctypes.c_int64 * 6)()
    n = rt.ggml_backend_mi355x_graph_stats_ex(be, arr, 6)
    assert n == 6
    return list(arr)


class ChainGraph:
    """x -> [add(., a_i) -> gelu -> scale(s_i)] x depth: 3 * depth kernels that node fusion keeps
    separate, built once and computed many times."""

    def __init__(self, rt, be, n=3072, rows=4, depth=4, scales=None):
        self.rt, self.be = rt, be
        ovh = rt.ggml_tensor_overhead() * (8 * depth + 8) + rt.ggml_graph_overhead()
        self.ctx = G.Context(rt, ovh, no_alloc=True)
        c = self.ctx.ctx
        self.x = rt.ggml_new_tensor_2d(c, F32, n, rows)
        self.a = [rt.ggml_new_tensor_1d(c, F32, n) for _ in range(depth)]
        cur = self.x
        scales = scales or [0.5 + 0.1 * i for i in range(depth)]
        for i in range(depth):
            cur = rt.ggml_add(c, cur, self.a[i])
            cur = rt.ggml_gelu(c, cur)
            cur = rt.ggml_scale(c, cur, scales[i])
        self.out = cur
        self.g = rt.ggml_new_graph(c)
        rt.ggml_build_forward_expand(self.g, self.out)
        self.buf = rt.ggml_backend_alloc_ctx_tensors(c, be)
        assert self.buf
        self.n, self.rows = n, rows
        for i, t in enumerate(self.a):
            G.tensor_set(rt, t, synth.uniform(100 + i, n))

    def run(self, seed):
        G.tensor_set(self.rt, self.x, synth.uniform(seed, self.n * self.rows) * np.float32(3.0))
        assert self.rt.ggml_backend_graph_compute(self.be, self.g) == G.GGML_STATUS_SUCCESS
        return G.tensor_get(self.rt, self.out)

    def free(self):
        self.rt.ggml_backend_buffer_free(self.buf)
        self.ctx.free()


def test_graph_compute_captures_and_replays_bit_identical():
    rt = G.runtime()
    direct_be = G.mi355x_backend(rt)
    be = G.mi355x_backend(rt)
    rt.ggml_backend_mi355x_set_graph_capture(direct_be, False)
    ref = ChainGraph(rt, direct_be)
    cg = ChainGraph(rt, be)
    try:
        s0 = _stats(rt, be)
        outs = [cg.run(seed) for seed in (1, 2, 3, 4)]
        s1 = _stats(rt, be)
        # run 1: direct (first graph of its topology), run 2: captured, runs 3-4: replays
        assert s1[3] - s0[3] == 1, (s0, s1)
        assert s1[5] - s0[5] == 1, (s0, s1)
        assert s1[4] - s0[4] == 2, (s0, s1)
        assert rt.ggml_backend_mi355x_last_launch_count(be) >= 4
        for seed, o in zip((1, 2, 3, 4), outs):
            r = ref.run(seed)
            assert np.array_equal(o.view(np.uint32), r.view(np.uint32)), seed
    finally:
        cg.free()
        ref.free()
        rt.ggml_backend_free(be)
        rt.ggml_backend_free(direct_be)


def test_graph_compute_updates_same_topology_in_place():
    """Graphs that differ only in a parameter (the scale op's factor) share a topology: the second
    one is captured and updates the first one's executable graph instead of instantiating."""
    rt = G.runtime()
    be = G.mi355x_backend(rt)
    direct_be = G.mi355x_backend(rt)
    rt.ggml_backend_mi355x_set_graph_capture(direct_be, False)
    graphs = [ChainGraph(rt, be, scales=[0.25 * (k + 1)] * 4) for k in range(3)]
    refs = [ChainGraph(rt, direct_be, scales=[0.25 * (k + 1)] * 4) for k in range(3)]
    try:
        graphs[0].run(7)  # direct: first of the topology
        s0 = _stats(rt, be)
        outs = [g.run(8) for g in graphs]  # capture + instantiate, then two captures + updates
        s1 = _stats(rt, be)
        assert s1[5] - s0[5] == 3 and s1[1] - s0[1] == 1 and s1[2] - s0[2] == 2, (s0, s1)
        outs2 = [g.run(9) for g in graphs]  # each graph's content is cached once: updated again
        for k in range(3):
            assert np.array_equal(outs[k].view(np.uint32), refs[k].run(8).view(np.uint32)), k
            assert np.array_equal(outs2[k].view(np.uint32), refs[k].run(9).view(np.uint32)), k
    finally:
        for g in graphs + refs:
            g.free()
        rt.ggml_backend_free(be)
        rt.ggml_backend_free(direct_be)


def test_graph_compute_capture_of_prefill_mul_mats():
    """Batched (prefill) mul_mats -- activation quantizer + int8 GEMM per node -- replayed from a
    capture give the direct launch's bits."""
    rt = G.runtime()
    be = G.mi355x_backend(rt)
    direct_be = G.mi355x_backend(rt)
    rt.ggml_backend_mi355x_set_graph_capture(direct_be, False)
    K, N, B = 1024, 512, 40
    outs = {}
    for name, b in (("capture", be), ("direct", direct_be)):
        ovh = rt.ggml_tensor_overhead() * 16 + rt.ggml_graph_overhead()
        ctx = G.Context(rt, ovh, no_alloc=True)
        c = ctx.ctx
        ws = [rt.ggml_new_tensor_2d(c, t, K, N) for t in (12, 13, 12)]
        x = rt.ggml_new_tensor_2d(c, F32, K, B)
        ys = [rt.ggml_mul_mat(c, w, x) for w in ws]
        g = rt.ggml_new_graph(c)
        for y in ys:
            rt.ggml_build_forward_expand(g, y)
        buf = rt.ggml_backend_alloc_ctx_tensors(c, b)
        try:
            for i, (w, t) in enumerate(zip(ws, (12, 13, 12))):
                wq = np.empty(G.row_size(t, K) * N, np.uint8)
                wf = synth.uniform(50 + i, K * N)
                rt.ggml_quantize_chunk(t, wf.ctypes.data, wq.ctypes.data, 0, N, K, None)
                G.tensor_set(rt, w, wq)
            res = []
            for seed in (1, 2, 3, 4):
                G.tensor_set(rt, x, synth.uniform(seed, K * B))
                assert rt.ggml_backend_graph_compute(b, g) == G.GGML_STATUS_SUCCESS
                res.append(np.concatenate([G.tensor_get(rt, y) for y in ys]))
            outs[name] = res
        finally:
            rt.ggml_backend_buffer_free(buf)
            ctx.free()
    st = _stats(rt, be)
    assert st[4] >= 2, st
    for a, d in zip(outs["capture"], outs["direct"]):
        assert np.array_equal(a.view(np.uint32), d.view(np.uint32))
    rt.ggml_backend_free(be)
    rt.ggml_backend_free(direct_be)
