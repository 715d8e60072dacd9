"""Kernel-duration sweep of the decode F16 GEMV (GPT-2 shapes) on MI355X.

Each config is one graph (optional norm->mul->add chain feeding mul_mat f16 [+ bias]) run ITERS
times; run under `rocprofv3 --kernel-trace` and pass the trace to --parse to get the per-config
average kernel duration (dispatches are attributed in order; the config list is printed first).
  python tools/micro_f16.py > order.json
  python tools/micro_f16.py --parse trace.csv order.json
"""
import json
import os
import sys

ITERS = 50
CONFIGS = []
for variant, threads in ((0, 0), (0, 64), (0, 256), (1, 0)):
    for (K, N, norm, rot) in ((768, 2304, 1, 1), (768, 3072, 1, 1), (768, 768, 0, 1), (3072, 768, 0, 1), (768, 50257, 1, 1),
                              (768, 2304, 0, 1), (768, 2304, 1, 16)):
        CONFIGS.append(dict(variant=variant, threads=threads, K=K, N=N, norm=norm, rot=rot))


def parse(trace, order):
    import csv
    cfgs = json.load(open(order))
    rows = list(csv.DictReader(open(trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = [r for r in rows if "k_mmv_f16" in r["Kernel_Name"] or "k_norm" in r["Kernel_Name"] or "k_convert" in r["Kernel_Name"]]
    i = 0
    for c in cfgs:
        n = c["dispatches"]
        seg = rows[i:i + n]
        i += n
        durs = sorted(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg[len(seg) // 5:])
        med = durs[len(durs) // 2] / 1e3 if durs else float("nan")
        name = seg[-1]["Kernel_Name"].split("(")[0][-40:] if seg else "?"
        print(f"v{c['variant']} t{c['threads']:3d} K={c['K']:5d} N={c['N']:6d} norm={c['norm']} rot={c['rot']:2d}  median {med:7.2f} us  "
              f"{c['K'] * c['N'] * 2 / (med * 1e-6) / 1e9 if durs else 0:7.0f} GB/s  {name}")


def main():
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ggml-imax_amd"))
    import numpy as np
    from ggml_mi355x import ggml as G, synth
    rt = G.runtime()
    be = G.mi355x_backend(rt)
    F32, F16 = G.GGML_TYPE_F32, G.GGML_TYPE_F16
    out_cfgs = []
    for cf in CONFIGS:
        rt.ggml_backend_mi355x_set_tuning(b"f16_variant", cf["variant"])
        rt.ggml_backend_mi355x_set_tuning(b"f16_threads", cf["threads"])
        K, N, R = cf["K"], cf["N"], cf["rot"]
        ctx = G.Context(rt, rt.ggml_tensor_overhead() * (16 + 8 * R) + R * rt.ggml_graph_overhead() + (1 << 20), no_alloc=True)
        c = ctx.ctx
        x = rt.ggml_new_tensor_2d(c, F32, K, 1)
        g = rt.ggml_new_tensor_1d(c, F32, K)
        b = rt.ggml_new_tensor_1d(c, F32, K)
        bias = rt.ggml_new_tensor_1d(c, F32, N)
        ws, graphs = [], []
        for r in range(R):
            w = rt.ggml_new_tensor_2d(c, F16, K, N)
            ws.append(w)
            h = rt.ggml_add(c, rt.ggml_mul(c, rt.ggml_norm(c, x, 1e-5), g), b) if cf["norm"] else x
            out = rt.ggml_add(c, rt.ggml_mul_mat(c, w, h), bias)
            gr = rt.ggml_new_graph(c)
            rt.ggml_build_forward_expand(gr, out)
            graphs.append(gr)
        buf = rt.ggml_backend_alloc_ctx_tensors(c, be)
        G.tensor_set(rt, x, synth.uniform(1, K))
        G.tensor_set(rt, g, synth.uniform(2, K) + np.float32(1))
        G.tensor_set(rt, b, synth.uniform(3, K))
        G.tensor_set(rt, bias, synth.uniform(5, N))
        wv = (synth.uniform(4, K * N) * 0.1).astype(np.float16)
        for w in ws:
            G.tensor_set(rt, w, wv)
        rt.ggml_backend_synchronize(be)
        launches = 0
        for it in range(ITERS):
            rt.ggml_backend_graph_compute_async(be, graphs[it % R])
            launches += rt.ggml_backend_mi355x_last_launch_count(be)
        rt.ggml_backend_synchronize(be)
        out_cfgs.append(dict(cf, dispatches=launches))
        rt.ggml_backend_buffer_free(buf)
        ctx.free()
    rt.ggml_backend_free(be)
    print(json.dumps(out_cfgs))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--parse":
        parse(sys.argv[2], sys.argv[3])
    else:
        main()
