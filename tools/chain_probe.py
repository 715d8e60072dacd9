"""Per-kernel cost of dependent chains of decode-shaped graph pieces on MI355X, replayed as one
graph plan (hipGraph): isolates a GEMV's body cost from the kernel-boundary floor.

  python tools/chain_probe.py [reps]
Each config is one ggml graph of L dependent pieces; the plan is computed `reps` times and the
wall time per piece is printed (host timer around plan_compute + synchronize)."""
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ggml-imax_amd"))
from ggml_mi355x import ggml as G, synth  # noqa: E402

F32, F16 = G.GGML_TYPE_F32, G.GGML_TYPE_F16


def build(rt, kind, L):
    ctx = G.Context(rt, rt.ggml_tensor_overhead() * (16 * L + 64) + rt.ggml_graph_overhead_custom(16 * L + 64, False), no_alloc=True)
    c = ctx.ctx
    E, F = 768, 3072
    x = rt.ggml_new_tensor_1d(c, F32, E)
    g = rt.ggml_new_tensor_1d(c, F32, E)
    b = rt.ggml_new_tensor_1d(c, F32, E)
    bE = rt.ggml_new_tensor_1d(c, F32, E)
    bF = rt.ggml_new_tensor_1d(c, F32, F)
    b3 = rt.ggml_new_tensor_1d(c, F32, 3 * E)
    ws, extra = [], []
    cur = x
    for i in range(L):
        if kind == "add":
            cur = rt.ggml_add(c, cur, bE)
        elif kind == "mm768":
            w = rt.ggml_new_tensor_2d(c, F16, E, E); ws.append(w)
            cur = rt.ggml_mul_mat(c, w, cur)
        elif kind == "mm768_bias_resid":
            w = rt.ggml_new_tensor_2d(c, F16, E, E); ws.append(w)
            cur = rt.ggml_add(c, rt.ggml_add(c, rt.ggml_mul_mat(c, w, cur), bE), cur)
        elif kind == "ln_mm768":
            w = rt.ggml_new_tensor_2d(c, F16, E, E); ws.append(w)
            h = rt.ggml_add(c, rt.ggml_mul(c, rt.ggml_norm(c, cur, 1e-5), g), b)
            cur = rt.ggml_add(c, rt.ggml_mul_mat(c, w, h), bE)
        elif kind == "mlp":  # LN + fc + bias + GELU, then proj + bias + resid (2 pieces)
            w1 = rt.ggml_new_tensor_2d(c, F16, E, F); w2 = rt.ggml_new_tensor_2d(c, F16, F, E); ws += [w1, w2]
            h = rt.ggml_add(c, rt.ggml_mul(c, rt.ggml_norm(c, cur, 1e-5), g), b)
            h = rt.ggml_gelu(c, rt.ggml_add(c, rt.ggml_mul_mat(c, w1, h), bF))
            cur = rt.ggml_add(c, rt.ggml_add(c, rt.ggml_mul_mat(c, w2, h), bE), cur)
        elif kind == "lm_head":  # ln_f + lm_head (768 x 50257), chained through the first 768 logits
            w = rt.ggml_new_tensor_2d(c, F16, E, 50257); ws.append(w)
            h = rt.ggml_add(c, rt.ggml_mul(c, rt.ggml_norm(c, cur, 1e-5), g), b)
            cur = rt.ggml_view_1d(c, rt.ggml_mul_mat(c, w, h), E, 0)
        elif kind == "c_attn":  # ln_1 + c_attn (768 x 2304) + bias + K/V cache row copies, chained through Q
            w = rt.ggml_new_tensor_2d(c, F16, E, 3 * E); ws.append(w)
            kc = rt.ggml_new_tensor_1d(c, F32, E); vc = rt.ggml_new_tensor_1d(c, F32, E)
            h = rt.ggml_add(c, rt.ggml_mul(c, rt.ggml_norm(c, cur, 1e-5), g), b)
            y = rt.ggml_add(c, rt.ggml_mul_mat(c, w, h), b3)
            extra += [rt.ggml_cpy(c, rt.ggml_view_1d(c, y, E, 4 * E), kc), rt.ggml_cpy(c, rt.ggml_view_1d(c, y, E, 8 * E), vc)]
            cur = rt.ggml_view_1d(c, y, E, 0)
        elif kind == "fc_gelu":
            w1 = rt.ggml_new_tensor_2d(c, F16, E, F); w2 = rt.ggml_new_tensor_2d(c, F16, F, E); ws += [w1, w2]
            h = rt.ggml_gelu(c, rt.ggml_add(c, rt.ggml_mul_mat(c, w1, cur), bF))
            cur = rt.ggml_mul_mat(c, w2, h)
    gr = rt.ggml_new_graph_custom(c, 16 * L + 64, False)
    for t in extra:
        rt.ggml_build_forward_expand(gr, t)
    rt.ggml_build_forward_expand(gr, cur)
    return ctx, gr, (x, g, b, bE, bF, b3), ws


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    rt = G.runtime()
    be = G.mi355x_backend(rt)
    only = sys.argv[2].split(",") if len(sys.argv) > 2 else None
    tunings = [t.split("=") for t in sys.argv[3].split(",")] if len(sys.argv) > 3 else [("f16_rgs", "0")]
    for kind, L, (tn, tv) in [(k, 4 if k == "lm_head" else 24, t)
                               for k in ("add", "mm768", "mm768_bias_resid", "ln_mm768", "c_attn", "fc_gelu", "mlp", "lm_head")
                               for t in tunings if not only or k in only]:
        rt.ggml_backend_mi355x_set_tuning(tn.encode(), int(tv))
        ctx, gr, vecs, ws = build(rt, kind, L)
        buf = rt.ggml_backend_alloc_ctx_tensors(ctx.ctx, be)
        for i, v in enumerate(vecs):
            n = rt.ggml_nelements(v)
            G.tensor_set(rt, v, (synth.uniform(100 + i, n) * 0.1 + (1.0 if i == 1 else 0.0)).astype(np.float32))
        for i, w in enumerate(ws):
            n = rt.ggml_nelements(w)
            G.tensor_set(rt, w, (synth.uniform(200 + i, n) * 0.05).astype(np.float16))
        res = {}
        for mode in ("plan", "eager"):
            rt.ggml_backend_mi355x_set_graph_capture(be, mode == "plan")
            plan = rt.ggml_backend_graph_plan_create(be, gr)
            for _ in range(5):
                rt.ggml_backend_graph_plan_compute(be, plan)
            rt.ggml_backend_synchronize(be)
            t0 = time.perf_counter()
            for _ in range(reps):
                rt.ggml_backend_graph_plan_compute(be, plan)
            rt.ggml_backend_synchronize(be)
            dt = time.perf_counter() - t0
            rt.ggml_backend_graph_plan_free(be, plan)
            res[mode] = dt / reps
        launches = rt.ggml_backend_mi355x_last_launch_count(be)
        print(f"{kind:18s} {tn}={tv} L={L}: {launches:3d} launches  plan {res['plan'] * 1e6 / launches:6.2f} us/launch "
              f"({res['plan'] * 1e6:7.1f} us/graph)   eager {res['eager'] * 1e6 / launches:6.2f} us/launch", flush=True)
        rt.ggml_backend_buffer_free(buf)
        ctx.free()
    rt.ggml_backend_mi355x_set_graph_capture(be, True)
    rt.ggml_backend_free(be)


if __name__ == "__main__":
    main()
