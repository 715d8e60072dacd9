"""Cold-weight GEMV latency: R independent (norm->)f16 GEMV+bias chains over distinct weights
(R x 3.5 MB > the 256 MB MALL), one graph; per-kernel durations from rocprofv3 kernel trace."""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ggml-imax_amd"))
from ggml_mi355x import ggml as G, synth

rt = G.runtime()
be = G.mi355x_backend(rt)
E, N = 768, int(os.environ.get("MC_N", "2304"))
R = int(os.environ.get("MC_R", "96"))
mode = sys.argv[1] if len(sys.argv) > 1 else "gemv"
F32, F16 = G.GGML_TYPE_F32, G.GGML_TYPE_F16
ctx = G.Context(rt, rt.ggml_tensor_overhead() * (12 * R + 8) + rt.ggml_graph_overhead_custom(16 * R + 16, False), no_alloc=True)
c = ctx.ctx
gr = rt.ggml_new_graph_custom(c, 16 * R + 16, False)
x = rt.ggml_new_tensor_2d(c, F32, E, 1)
g = rt.ggml_new_tensor_1d(c, F32, E)
b = rt.ggml_new_tensor_1d(c, F32, E)
ws, bs = [], []
for r in range(R):
    w = rt.ggml_new_tensor_2d(c, F16, E, N); ws.append(w)
    bias = rt.ggml_new_tensor_1d(c, F32, N); bs.append(bias)
    h = rt.ggml_add(c, rt.ggml_mul(c, rt.ggml_norm(c, x, 1e-5), g), b) if mode == "normgemv" else x
    out = rt.ggml_add(c, rt.ggml_mul_mat(c, w, h), bias)
    rt.ggml_build_forward_expand(gr, out)
buf = rt.ggml_backend_alloc_ctx_tensors(c, be)
G.tensor_set(rt, x, synth.uniform(1, E))
G.tensor_set(rt, g, synth.uniform(2, E) + np.float32(1))
G.tensor_set(rt, b, synth.uniform(3, E))
wv = synth.uniform(4, E * N).astype(np.float16)
for r in range(R):
    G.tensor_set(rt, ws[r], wv)
    G.tensor_set(rt, bs[r], synth.uniform(5, N))
for _ in range(3):
    rt.ggml_backend_graph_compute(be, gr)
t0 = time.perf_counter()
for _ in range(10):
    rt.ggml_backend_graph_compute_async(be, gr)
rt.ggml_backend_synchronize(be)
print(mode, "N", N, "R", R, "us per chain", (time.perf_counter() - t0) / 10 / R * 1e6, "launches/graph", rt.ggml_backend_mi355x_last_launch_count(be))
