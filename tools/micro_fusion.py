"""Micro-benchmark of fused vs unfused GPT-2 blocks (norm->mul->add->mul_mat f16 [+bias]) on MI355X.
usage: python tools/micro_fusion.py  (set GGML_MI355X_NO_NODE_FUSION=1 for the unfused path)"""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ggml-imax_amd"))
from ggml_mi355x import ggml as G, synth

rt = G.runtime()
be = G.mi355x_backend(rt)
E, N, B = 768, 2304, 1
F32, F16 = G.GGML_TYPE_F32, G.GGML_TYPE_F16
ctx = G.Context(rt, rt.ggml_tensor_overhead() * 32 + rt.ggml_graph_overhead(), no_alloc=True)
c = ctx.ctx
x = rt.ggml_new_tensor_2d(c, F32, E, B)
g = rt.ggml_new_tensor_1d(c, F32, E)
b = rt.ggml_new_tensor_1d(c, F32, E)
w = rt.ggml_new_tensor_2d(c, F16, E, N)
bias = rt.ggml_new_tensor_1d(c, F32, N)
mode = sys.argv[1] if len(sys.argv) > 1 else "normgemv"
if mode == "normgemv":
    h = rt.ggml_add(c, rt.ggml_mul(c, rt.ggml_norm(c, x, 1e-5), g), b)
    out = rt.ggml_add(c, rt.ggml_mul_mat(c, w, h), bias)
elif mode == "gemv":
    out = rt.ggml_add(c, rt.ggml_mul_mat(c, w, x), bias)
else:
    out = rt.ggml_add(c, rt.ggml_mul(c, rt.ggml_norm(c, x, 1e-5), g), b)
gr = rt.ggml_new_graph(c)
rt.ggml_build_forward_expand(gr, out)
buf = rt.ggml_backend_alloc_ctx_tensors(c, be)
G.tensor_set(rt, x, synth.uniform(1, E * B))
G.tensor_set(rt, g, synth.uniform(2, E) + np.float32(1))
G.tensor_set(rt, b, synth.uniform(3, E))
G.tensor_set(rt, w, synth.uniform(4, E * N).astype(np.float16))
G.tensor_set(rt, bias, synth.uniform(5, N))
for _ in range(10):
    rt.ggml_backend_graph_compute(be, gr)
t0 = time.perf_counter()
for _ in range(200):
    rt.ggml_backend_graph_compute_async(be, gr)
rt.ggml_backend_synchronize(be)
print(mode, "us/graph", (time.perf_counter() - t0) / 200 * 1e6, "launches", rt.ggml_backend_mi355x_last_launch_count(be))
