"""Device timeline of the decode kernels from their phase stamps (diagnostic build: make -C
ggml-imax_amd diaglib; this script points GGML_MI355X_BACKEND_LIB at it).

  python tools/stamps.py lone q4_K:4096:4096:1 [...]   one mul_mat per graph, per-launch phases
  python tools/stamps.py gpt2 [f16|q4_k] [tokens]      GPT-2 decode: the last token's launches

Each instrumented workgroup records s_memrealtime (100 MHz: 10 ns ticks) in 8 slots: 0 entry,
7 exit, 1-4 kernel-specific phases (k_mmv_stream: 1 wave 0's activation slices quantized, 2 after
the workgroup barrier, 3 first row stored; k_gemv_f16: 1 activations staged, 3 dots done;
k_gemv_f16_ps: 1 parts summed, 2 after the barrier, 4 normalized; k_attn_proj: 1 head's attention
done). Per launch: span = last exit - first entry, the entry spread, the gap to the previous
launch's last exit, and per-workgroup medians of the phases."""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("GGML_MI355X_BACKEND_LIB", os.path.join(REPO, "ggml-imax_amd", "lib", "diag", "libggml_mi355x.so"))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "ggml-imax_amd"))
from ggml_mi355x import ggml as G  # noqa: E402

SLOTS = 8 << 20
TICK_US = 0.01


def read(lib):
    words = np.zeros(SLOTS, np.uint64)
    log = ctypes.create_string_buffer(1 << 22)
    n = lib.ggml_backend_mi355x_stamps_read(words.ctypes.data, SLOTS, log, len(log))
    launches = []
    for line in log.value.decode().splitlines():
        name, nb, off = line.split()
        nb, off = int(nb), int(off)
        st = words[off:off + 8 * nb].reshape(nb, 8).astype(np.int64)
        if st[:, 0].min() == 0 or st[:, 7].min() == 0:
            continue  # not executed (a capture that never replayed) or overwritten
        launches.append((name, nb, st))
    launches.sort(key=lambda L: L[2][:, 0].min())
    return n, launches


def phase(st, a, b):
    m = (st[:, a] > 0) & (st[:, b] > 0)
    return float(np.median(st[m, b] - st[m, a])) * TICK_US if m.any() else float("nan")


def report(launches, title):
    print(title)
    print(f"{'kernel':18s} {'WGs':>5s} {'gap':>6s} {'span':>6s} {'spread':>6s} {'wg_med':>6s} {'wg_max':>6s}  phases (median us)")
    prev_end = None
    tot_span = tot_gap = 0.0
    for name, nb, st in launches:
        t0, t7 = st[:, 0], st[:, 7]
        span = (t7.max() - t0.min()) * TICK_US
        gap = (t0.min() - prev_end) * TICK_US if prev_end is not None else 0.0
        prev_end = t7.max()
        tot_span += span
        tot_gap += gap
        wg = (t7 - t0) * TICK_US
        ph = " ".join(f"{a}->{b}:{phase(st, a, b):.2f}" for a, b in ((0, 1), (1, 2), (0, 2), (2, 1), (2, 3), (0, 3), (3, 4), (3, 7), (1, 4), (4, 1), (4, 7))
                      if not np.isnan(phase(st, a, b)) and 0 <= phase(st, a, b) < 1e4)
        # norm prologue (k_mmv_stream PRO): realtime slots 6 (mean certified), 5 (scale) instead of the clock
        rt = (st[:, 6] > st[:, 0]) & (st[:, 6] - st[:, 0] < 10**5) & (st[:, 5] >= st[:, 6]) & (st[:, 5] - st[:, 6] < 10**5)
        if rt.sum() > len(st) // 2:
            ph += " | norm: " + " ".join(f"{a}->{b}:{phase(st[rt], a, b):.2f}" for a, b in ((0, 6), (6, 5), (5, 2)))
            m = np.zeros(len(st), bool)
        else:
            m = (st[:, 5] > st[:, 6]) & (st[:, 7] > st[:, 0]) & (st[:, 6] > 0)
        if m.any():  # shader clock: memtime ticks / realtime ticks x 100 MHz
            ph += f" clk:{np.median((st[m, 5] - st[m, 6]) / (st[m, 7] - st[m, 0])) * 100:.0f}MHz"
        print(f"{name:18s} {nb:5d} {gap:6.2f} {span:6.2f} {(t0.max() - t0.min()) * TICK_US:6.2f} {np.median(wg):6.2f} {wg.max():6.2f}  {ph}")
    print(f"launches {len(launches)}: sum of spans {tot_span:.1f} us, sum of gaps {tot_gap:.1f} us, "
          f"first entry -> last exit {(launches[-1][2][:, 7].max() - launches[0][2][:, 0].min()) * TICK_US:.1f} us")


def lone(cases):
    import bench
    lib = G.runtime()
    assert lib.ggml_backend_mi355x_stamps_enable(SLOTS), "stamps need the diagnostic build (make -C ggml-imax_amd diaglib)"
    be = G.mi355x_backend(lib)
    for case in cases:
        tn, K, N, B = case.split(":")
        t, K, N, B = bench.TYPE_NAMES[tn], int(K), int(N), int(B)
        R = max(8, int(320 * 2**20 // (G.row_size(t, K) * N)) + 1)
        w = bench.RotatedSingle(lib, be, t, K, N, B, R)
        for _ in range(2 * R):
            w.step()
        lib.ggml_backend_synchronize(be)
        lib.ggml_backend_mi355x_stamps_reset()
        for _ in range(6):
            w.step()
        lib.ggml_backend_synchronize(be)
        _, L = read(lib)
        report(L, f"== {case}: 6 graphs, one mul_mat each")
        w.free()
    lib.ggml_backend_free(be)


def gpt2_run(kind, n_tok):
    from ggml_mi355x import gpt2
    lib = G.runtime()
    assert lib.ggml_backend_mi355x_stamps_enable(SLOTS), "stamps need the diagnostic build (make -C ggml-imax_amd diaglib)"
    be = G.mi355x_backend(lib)
    path = gpt2.ensure_model() if kind == "f16" else gpt2.ensure_quantized_model(lib, kind)
    m = gpt2.Model(lib, path, be, n_ctx=1024, n_batch=8)
    toks = m.tokenize("Once upon a time the cat sat on the mat and the dog ran away")[:32]
    n_past = 0
    for i in range(0, len(toks), 8):
        lg = m.eval(n_past, toks[i:i + 8])
        n_past += len(toks[i:i + 8])
    nxt = int(np.argmax(lg[-1]))
    lib.ggml_backend_mi355x_stamps_reset()
    for _ in range(n_tok):
        lg = m.eval(n_past, [nxt], copy=False)
        n_past += 1
        nxt = int(np.argmax(lg[-1]))
    lib.ggml_backend_synchronize(be)
    _, L = read(lib)
    per = lib.ggml_backend_mi355x_last_launch_count(be)
    # launches of the last token: the stamped kernels since the last embedding launch
    last = max(i for i, x in enumerate(L) if x[0] == "k_get_rows_add")
    report(L[last:], f"== GPT-2 {kind} decode, last of {n_tok} tokens ({per} launches per token, stamped kernels listed)")
    if last > 0:
        prev = max(i for i, x in enumerate(L[:last]) if x[0] == "k_get_rows_add")
        tok = (L[last][2][:, 0].min() - L[prev][2][:, 0].min()) * TICK_US
        print(f"token period (embedding entry to embedding entry): {tok:.1f} us")
    m.free()
    lib.ggml_backend_free(be)


def normgemv(E, N, B, reps=6):
    """norm -> mul(g) -> add(b) -> F16 mul_mat [E, N] x B columns -> add(bias): the fused F16 GEMV with
    its norm prologue (GPT-2's c_attn / c_fc shape), one graph per step over rotated weights"""
    from ggml_mi355x import synth
    lib = G.runtime()
    assert lib.ggml_backend_mi355x_stamps_enable(SLOTS), "stamps need the diagnostic build"
    be = G.mi355x_backend(lib)
    R = 24
    ctx = G.Context(lib, lib.ggml_tensor_overhead() * (8 * R + 8) + lib.ggml_graph_overhead_custom(16, False) * R, no_alloc=True)
    c = ctx.ctx
    x = lib.ggml_new_tensor_2d(c, G.GGML_TYPE_F32, E, B)
    g = lib.ggml_new_tensor_1d(c, G.GGML_TYPE_F32, E)
    b = lib.ggml_new_tensor_1d(c, G.GGML_TYPE_F32, E)
    graphs, ws = [], []
    for r in range(R):
        w = lib.ggml_new_tensor_2d(c, G.GGML_TYPE_F16, E, N)
        bias = lib.ggml_new_tensor_1d(c, G.GGML_TYPE_F32, N)
        h = lib.ggml_add(c, lib.ggml_mul(c, lib.ggml_norm(c, x, 1e-5), g), b)
        out = lib.ggml_add(c, lib.ggml_mul_mat(c, w, h), bias)
        gr = lib.ggml_new_graph_custom(c, 16, False)
        lib.ggml_build_forward_expand(gr, out)
        graphs.append(gr)
        ws.append((w, bias))
    buf = lib.ggml_backend_alloc_ctx_tensors(c, be)
    G.tensor_set(lib, x, synth.uniform(1, E * B))
    G.tensor_set(lib, g, synth.uniform(2, E) + np.float32(1))
    G.tensor_set(lib, b, synth.uniform(3, E))
    wv = synth.uniform(4, E * N).astype(np.float16)
    for w, bias in ws:
        G.tensor_set(lib, w, wv)
        G.tensor_set(lib, bias, synth.uniform(5, N))
    for gr in graphs:
        lib.ggml_backend_graph_compute(be, gr)
    lib.ggml_backend_mi355x_stamps_reset()
    for i in range(reps):
        lib.ggml_backend_graph_compute_async(be, graphs[i % R])
    lib.ggml_backend_synchronize(be)
    _, L = read(lib)
    report(L, f"== norm -> F16 GEMV {E}x{N}, {B} columns")
    lib.ggml_backend_buffer_free(buf)
    ctx.free()
    lib.ggml_backend_free(be)


def f16gemv(K, N, B, reps=6):
    """F16 mul_mat [K, N] x B columns -> add(bias) -> add(residual): GPT-2's MLP c_proj shape, no
    prologue, one graph per step over rotated weights"""
    from ggml_mi355x import synth
    lib = G.runtime()
    assert lib.ggml_backend_mi355x_stamps_enable(SLOTS), "stamps need the diagnostic build"
    be = G.mi355x_backend(lib)
    R = 24
    ctx = G.Context(lib, lib.ggml_tensor_overhead() * (8 * R + 8) + lib.ggml_graph_overhead_custom(16, False) * R, no_alloc=True)
    c = ctx.ctx
    x = lib.ggml_new_tensor_2d(c, G.GGML_TYPE_F32, K, B)
    res = lib.ggml_new_tensor_2d(c, G.GGML_TYPE_F32, N, B)
    graphs, ws = [], []
    for r in range(R):
        w = lib.ggml_new_tensor_2d(c, G.GGML_TYPE_F16, K, N)
        bias = lib.ggml_new_tensor_1d(c, G.GGML_TYPE_F32, N)
        out = lib.ggml_add(c, lib.ggml_add(c, lib.ggml_mul_mat(c, w, x), bias), res)
        gr = lib.ggml_new_graph_custom(c, 16, False)
        lib.ggml_build_forward_expand(gr, out)
        graphs.append(gr)
        ws.append((w, bias))
    buf = lib.ggml_backend_alloc_ctx_tensors(c, be)
    G.tensor_set(lib, x, synth.uniform(1, K * B))
    G.tensor_set(lib, res, synth.uniform(2, N * B))
    wv = synth.uniform(4, K * N).astype(np.float16)
    for w, bias in ws:
        G.tensor_set(lib, w, wv)
        G.tensor_set(lib, bias, synth.uniform(5, N))
    for gr in graphs:
        lib.ggml_backend_graph_compute(be, gr)
    lib.ggml_backend_mi355x_stamps_reset()
    for i in range(reps):
        lib.ggml_backend_graph_compute_async(be, graphs[i % R])
    lib.ggml_backend_synchronize(be)
    _, L = read(lib)
    report(L, f"== F16 GEMV {K}x{N} + bias + residual, {B} columns")
    lib.ggml_backend_buffer_free(buf)
    ctx.free()
    lib.ggml_backend_free(be)


if __name__ == "__main__":
    if sys.argv[1] == "f16gemv":
        f16gemv(int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]))
        sys.exit(0)
    if sys.argv[1] == "normgemv":
        normgemv(int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]))
        sys.exit(0)
    if sys.argv[1] == "lone":
        lone(sys.argv[2:] or ["q4_K:4096:4096:1"])
    else:
        gpt2_run(sys.argv[2] if len(sys.argv) > 2 else "f16", int(sys.argv[3]) if len(sys.argv) > 3 else 8)
