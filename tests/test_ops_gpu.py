"""Companion ops at GPT-2 / LLaMA shapes vs the reference CPU backend
(oracle/_ref/libggml_ref.so) itself, bit for bit where the CPU's rounding sequence is reproducible.

The reference's test-backend-ops (tests/test_00_reference_harness.py) checks these ops with NMSE
thresholds; here the same graphs run on MI355X and on the reference CPU and the outputs must be
identical bits: norms and soft_max run the CPU's sequential double sums, lookup tables are built
with the reference build's own contraction choices, and no multiply-add is fused unless the CPU
fuses it. RoPE is exact where the backend's host-built cos/sin table covers the position.
"""
import os

import numpy as np
import pytest

from conftest import REPO
from ggml_mi355x import ggml as G
from ggml_mi355x import synth

REF_LIB = os.path.join(REPO, "oracle", "_ref", "libggml_ref.so")

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not os.path.exists(REF_LIB), reason="make -C oracle ref")]

F32, F16, I32 = G.GGML_TYPE_F32, G.GGML_TYPE_F16, G.GGML_TYPE_I32


@pytest.fixture(scope="module")
def libs():
    rt = G.runtime()
    be = G.mi355x_backend(rt)
    ref = G.Lib([REF_LIB], isolated=True)
    cpu = ref.ggml_backend_cpu_init()
    yield rt, be, ref, cpu
    ref.ggml_backend_free(cpu)
    rt.ggml_backend_free(be)


def both(libs, build):
    rt, be, ref, cpu = libs
    return G.graph_once(rt, be, lambda c: build(rt, c)), G.graph_once(ref, cpu, lambda c: build(ref, c))


def ulp_diff(a, b):
    ai = a.view(np.int32).astype(np.int64)
    bi = b.view(np.int32).astype(np.int64)
    return np.abs(ai - bi)


def assert_exact(a, b, name, allow_ulp1_frac=0.0):
    assert a.shape == b.shape
    fin = np.isfinite(b)
    assert np.array_equal(np.isfinite(a), fin), f"{name}: inf/nan pattern differs"
    d = ulp_diff(a[fin], b[fin])
    n_bad = int(np.sum(d > 0))
    print(f"{name}: {n_bad}/{d.size} elements differ (max {int(d.max()) if d.size else 0} ulp)")
    if allow_ulp1_frac == 0.0:
        assert n_bad == 0
    else:
        assert int(d.max()) <= 1 and n_bad <= allow_ulp1_frac * d.size


def rnd(seed, n, scale=1.0):
    return (synth.uniform(seed, n) * np.float32(scale)).astype(np.float32)


@pytest.mark.parametrize("ne0,ne1", [(768, 1), (768, 8), (3072, 5), (4096, 3)])
def test_norm_exact(libs, ne0, ne1):
    x = rnd(1, ne0 * ne1, 3.0) + np.float32(0.5)

    def build(L, c):
        t = L.ggml_new_tensor_2d(c, F32, ne0, ne1)
        return [(t, x)], L.ggml_norm(c, t, 1e-5)

    a, b = both(libs, build)
    assert_exact(a, b, "norm")


def test_norm_tie_rows_take_sequential_path(libs):
    """Rows whose mean sits exactly on a float rounding midpoint: the certified parallel path
    cannot decide them and the kernel must replay the CPU's sequential double sum."""
    rows = []
    for k in range(16):
        r = np.zeros(8, np.float32)
        r[0] = np.float32(1.0 + k * 2.0**-20)
        r[1] = np.float32(2.0**-24)   # sum/8 = 0.125 + 2^-27: halfway between two floats
        r[2 + k % 6] = np.float32(-(2.0**-30)) if k % 2 else np.float32(0.0)
        rows.append(r)
    x = np.concatenate(rows)

    def build(L, c):
        t = L.ggml_new_tensor_2d(c, F32, 8, 16)
        return [(t, x)], L.ggml_norm(c, t, 1e-5)

    a, b = both(libs, build)
    assert_exact(a, b, "norm (tie rows)")


@pytest.mark.parametrize("ne0,ne1", [(4096, 1), (4096, 7)])
def test_rms_norm_exact(libs, ne0, ne1):
    x = rnd(2, ne0 * ne1, 2.0)

    def build(L, c):
        t = L.ggml_new_tensor_2d(c, F32, ne0, ne1)
        return [(t, x)], L.ggml_rms_norm(c, t, 1e-6)

    a, b = both(libs, build)
    assert_exact(a, b, "rms_norm")


@pytest.mark.parametrize("n_kv,N", [(1, 1), (13, 1), (40, 8), (1000, 1), (512, 16)])
def test_gpt2_attention_softmax_exact(libs, n_kv, N):
    """scale -> diag_mask_inf(n_past) -> soft_max as in gpt2_graph (main-backend.cpp:572-584)."""
    H = 12
    n_past = n_kv - N
    x = rnd(3, n_kv * N * H, 4.0)

    def build(L, c):
        t = L.ggml_new_tensor_3d(c, F32, n_kv, N, H)
        s = L.ggml_scale(c, t, 1.0 / 8.0)
        m = L.ggml_diag_mask_inf(c, s, n_past)
        return [(t, x)], L.ggml_soft_max(c, m)

    a, b = both(libs, build)
    assert_exact(a, b, "scale+diag_mask_inf+soft_max")


def test_gelu_exact(libs):
    # every f16 input value of the lookup table plus the clamp regions
    h = np.arange(65536, dtype=np.uint16).view(np.float16).astype(np.float32)
    h = h[np.isfinite(h)]
    x = np.concatenate([h, rnd(4, 30000, 12.0)]).astype(np.float32)

    def build(L, c):
        t = L.ggml_new_tensor_1d(c, F32, len(x))
        return [(t, x)], L.ggml_gelu(c, t)

    a, b = both(libs, build)
    assert_exact(a, b, "gelu")


def test_silu_exact(libs):
    x = rnd(5, 50000, 9.0)

    def build(L, c):
        t = L.ggml_new_tensor_1d(c, F32, len(x))
        return [(t, x)], L.ggml_silu(c, t)

    a, b = both(libs, build)
    assert_exact(a, b, "silu")


@pytest.mark.parametrize("src_type", [F16, F32])
def test_get_rows_plus_add_exact(libs, src_type):
    """get_rows(wte f16) + get_rows(wpe f32) as the GPT-2 embedding (main-backend.cpp:475-478)."""
    E, V, N = 768, 997, 9
    w = rnd(6, E * V, 0.1)
    wv = w.astype(np.float16) if src_type == F16 else w
    p = rnd(7, E * 64, 0.1)
    ids = np.array([5, 996, 0, 17, 17, 300, 2, 9, 500], dtype=np.int32)
    pos = np.arange(N, dtype=np.int32) + 3

    def build(L, c):
        wt = L.ggml_new_tensor_2d(c, src_type, E, V)
        pt = L.ggml_new_tensor_2d(c, F32, E, 64)
        it = L.ggml_new_tensor_1d(c, I32, N)
        qt = L.ggml_new_tensor_1d(c, I32, N)
        out = L.ggml_add(c, L.ggml_get_rows(c, wt, it), L.ggml_get_rows(c, pt, qt))
        return [(wt, wv), (pt, p), (it, ids), (qt, pos)], out

    a, b = both(libs, build)
    assert_exact(a, b, "get_rows+add")


@pytest.mark.parametrize("qtype", [G.GGML_TYPE_Q4_0, G.GGML_TYPE_Q8_0, G.GGML_TYPE_Q4_K, G.GGML_TYPE_Q5_K])
def test_get_rows_quantized_exact(libs, qtype):
    """get_rows of a quantized wte (a quantized GPT-2's embedding, ggml.c:12874-12918 dequantizes the
    picked rows with the type's to_float) + get_rows(wpe f32): identical bits."""
    import pyoracle as orc
    E, V, N = 768, 997, 9
    wq = orc.quantize(qtype, rnd(16, E * V, 0.1), E)
    p = rnd(7, E * 64, 0.1)
    ids = np.array([5, 996, 0, 17, 17, 300, 2, 9, 500], dtype=np.int32)
    pos = np.arange(N, dtype=np.int32) + 3

    def build(L, c):
        wt = L.ggml_new_tensor_2d(c, qtype, E, V)
        pt = L.ggml_new_tensor_2d(c, F32, E, 64)
        it = L.ggml_new_tensor_1d(c, I32, N)
        qt = L.ggml_new_tensor_1d(c, I32, N)
        out = L.ggml_add(c, L.ggml_get_rows(c, wt, it), L.ggml_get_rows(c, pt, qt))
        return [(wt, wq), (pt, p), (it, ids), (qt, pos)], out

    a, b = both(libs, build)
    assert_exact(a, b, f"get_rows(type {qtype})+add")
    # and the picked rows alone against the oracle's dequantization
    rt, be, _, _ = libs

    def build_rows(c):
        wt = rt.ggml_new_tensor_2d(c, qtype, E, V)
        it = rt.ggml_new_tensor_1d(c, I32, N)
        return [(wt, wq), (it, ids)], rt.ggml_get_rows(c, wt, it)

    rows = G.graph_once(rt, be, build_rows).reshape(N, E)
    deq = orc.dequantize(qtype, wq, E * V).reshape(V, E)[ids]
    assert np.array_equal(rows.view(np.uint32), deq.view(np.uint32))


def test_layernorm_affine_exact(libs):
    """norm -> mul(g) -> add(b) with row broadcast, as every GPT-2 layer norm."""
    E, N = 768, 6
    x = rnd(8, E * N, 2.0)
    g = rnd(9, E, 1.0) + np.float32(1.0)
    bb = rnd(10, E, 0.1)

    def build(L, c):
        t = L.ggml_new_tensor_2d(c, F32, E, N)
        gt = L.ggml_new_tensor_1d(c, F32, E)
        bt = L.ggml_new_tensor_1d(c, F32, E)
        return [(t, x), (gt, g), (bt, bb)], L.ggml_add(c, L.ggml_mul(c, L.ggml_norm(c, t, 1e-5), gt), bt)

    a, b = both(libs, build)
    assert_exact(a, b, "norm+mul+add")


def test_permute_cont_cpy_exact(libs):
    """cont(permute(reshape)) of the V cache (main-backend.cpp:586-594) and f32 -> f16 cpy."""
    D, H, T = 64, 12, 37
    x = rnd(11, D * H * T, 1.0)

    def build(L, c):
        t = L.ggml_new_tensor_3d(c, F32, D, H, T)
        p = L.ggml_cont(c, L.ggml_permute(c, t, 1, 2, 0, 3))
        h = L.ggml_new_tensor_3d(c, F16, T, D, H)
        return [(t, x)], L.ggml_cpy(c, p, h)

    a, b = both(libs, build)
    assert np.array_equal(a.view(np.uint16), b.view(np.uint16))


@pytest.mark.parametrize("order", [1, 0])
@pytest.mark.parametrize("n_past,N", [(0, 1), (5, 1), (39, 8), (100, 28), (200, 1), (300, 1), (990, 10), (0, 512)])
def test_gpt2_attention_block_exact(libs, n_past, N, order):
    """The whole attention block of gpt2_graph (main-backend.cpp:532-608): Q/K/V views of the
    c_attn output, K/V cache writes, cont/permute, KQ, scale, diag_mask_inf, soft_max, V_trans,
    KQV, merge. On MI355X it runs as one fused kernel: with mmv_order=1 (k_attn_fast /
    k_attn_ordered, the reference's summation order) bits must match the CPU; in the default
    order (k_attn_tree: f32 tree sums, same fp16 soft_max weights) within 5e-5 of max |out| (the
    outputs are weighted means of up to 1000 values: f32 summation-order error of either side)."""
    E, H, n_ctx = 768, 12, 1024
    D = E // H
    cur_v = rnd(13, 3 * E * N, 1.0)
    mem_k = rnd(14, E * n_ctx, 1.0)
    mem_v = rnd(15, E * n_ctx, 1.0)

    def build(L, c):
        cur = L.ggml_new_tensor_2d(c, F32, 3 * E, N)
        mk = L.ggml_new_tensor_1d(c, F32, E * n_ctx)
        mv = L.ggml_new_tensor_1d(c, F32, E * n_ctx)
        nb1 = cur.contents.nb[1]
        Qcur = L.ggml_view_2d(c, cur, E, N, nb1, 0)
        Kcur = L.ggml_view_2d(c, cur, E, N, nb1, 4 * E)
        Vcur = L.ggml_view_2d(c, cur, E, N, nb1, 8 * E)
        k = L.ggml_view_1d(c, mk, N * E, 4 * E * n_past)
        v = L.ggml_view_1d(c, mv, N * E, 4 * E * n_past)
        ck = L.ggml_cpy(c, Kcur, k)
        cv = L.ggml_cpy(c, Vcur, v)
        Q = L.ggml_permute(c, L.ggml_cont_3d(c, Qcur, D, H, N), 0, 2, 1, 3)
        K = L.ggml_permute(c, L.ggml_reshape_3d(c, L.ggml_view_1d(c, mk, (n_past + N) * E, 0), D, H, n_past + N), 0, 2, 1, 3)
        KQ = L.ggml_mul_mat(c, K, Q)
        sm = L.ggml_soft_max(c, L.ggml_diag_mask_inf(c, L.ggml_scale(c, KQ, 1.0 / np.sqrt(D)), n_past))
        Vt = L.ggml_cont_3d(c, L.ggml_permute(c, L.ggml_reshape_3d(c, L.ggml_view_1d(c, mv, (n_past + N) * E, 0), D, H, n_past + N),
                                              1, 2, 0, 3), n_past + N, D, H)
        KQV = L.ggml_mul_mat(c, Vt, sm)
        out = L.ggml_cont_2d(c, L.ggml_permute(c, KQV, 0, 2, 1, 3), E, N)
        return [(cur, cur_v), (mk, mem_k), (mv, mem_v)], (out, [ck, cv])

    rt, be, ref, cpu = libs

    def run(L, b):
        def bld(c):
            feeds, (out, extra) = build(L, c)
            return feeds, out, extra
        return graph_once_multi(L, b, bld)

    assert rt.ggml_backend_mi355x_set_tuning(b"mmv_order", order)
    try:
        a = run(rt, be)
    finally:
        rt.ggml_backend_mi355x_set_tuning(b"mmv_order", -1)
    b = run(ref, cpu)
    if order:
        assert_exact(a, b, "attention block")
    else:
        err = float(np.max(np.abs(a - b)) / np.max(np.abs(b)))
        print(f"attention block (tree order): rel err {err:.2e}")
        assert err <= 5e-5, err


def graph_once_multi(lib, backend, build, n_tensors=96):
    """graph_once with extra nodes expanded before the output (the K/V cache copies)."""
    overhead = lib.ggml_tensor_overhead() * n_tensors + lib.ggml_graph_overhead()
    with G.Context(lib, overhead, no_alloc=True) as c:
        feeds, out, extra = build(c.ctx)
        g = lib.ggml_new_graph(c.ctx)
        for e in extra:
            lib.ggml_build_forward_expand(g, e)
        lib.ggml_build_forward_expand(g, out)
        buf = lib.ggml_backend_alloc_ctx_tensors(c.ctx, backend)
        try:
            for t, arr in feeds:
                G.tensor_set(lib, t, arr)
            assert lib.ggml_backend_graph_compute(backend, g) == G.GGML_STATUS_SUCCESS
            return G.tensor_get(lib, out)
        finally:
            lib.ggml_backend_buffer_free(buf)


@pytest.mark.parametrize("mode", [0, 2])
def test_rope_exact(libs, mode):
    """RoPE (LLaMA mode 0, NeoX mode 2): bit-identical to the reference CPU for positions the
    backend's host-built {cos, sin} table covers (the reference's running theta product and the
    host libm's sincosf; NeoX's pair combined with the fma the reference build uses); positions
    past the table (here 5000 > 4096) use the device's own cos/sin: within 1e-5."""
    D, H, T = 128, 8, 12
    x = rnd(12, D * H * T, 1.0)
    pos = (np.arange(T, dtype=np.int32) * 37 + 5).astype(np.int32)
    pos[-1] = 5000

    def build(L, c):
        t = L.ggml_new_tensor_3d(c, F32, D, H, T)
        pt = L.ggml_new_tensor_1d(c, I32, T)
        return [(t, x), (pt, pos)], L.ggml_rope(c, t, pt, D, mode, 0)

    a, b = both(libs, build)
    a, b = a.reshape(T, H, D), b.reshape(T, H, D)
    d = ulp_diff(a, b)
    print(f"rope mode {mode}: {int(np.sum(d[:-1] > 0))}/{d[:-1].size} differ in the table, past it max abs "
          f"{float(np.max(np.abs(a[-1] - b[-1]))):.2e}")
    assert_exact(a[:-1], b[:-1], f"rope mode {mode}")
    assert np.max(np.abs(a[-1] - b[-1])) <= 1e-5 * max(1.0, float(np.max(np.abs(b[-1]))))


def graph_outputs(lib, backend, build, n_tensors=128):
    """Builds (feeds, outs, extra) in one context, computes once, returns every output's values and
    the backend's launch count."""
    overhead = lib.ggml_tensor_overhead() * n_tensors + lib.ggml_graph_overhead()
    with G.Context(lib, overhead, no_alloc=True) as c:
        feeds, outs, extra = build(c.ctx)
        g = lib.ggml_new_graph(c.ctx)
        for e in extra:
            lib.ggml_build_forward_expand(g, e)
        for o in outs:
            lib.ggml_build_forward_expand(g, o)
        buf = lib.ggml_backend_alloc_ctx_tensors(c.ctx, backend)
        try:
            for t, arr in feeds:
                G.tensor_set(lib, t, arr)
            assert lib.ggml_backend_graph_compute(backend, g) == G.GGML_STATUS_SUCCESS
            n = lib.ggml_backend_mi355x_last_launch_count(backend) if hasattr(lib, "ggml_backend_mi355x_last_launch_count") else 0
            return [G.tensor_get(lib, o) for o in outs], n
        finally:
            lib.ggml_backend_buffer_free(buf)


@pytest.mark.parametrize("consumer", ["ln_fc", "add"])
@pytest.mark.parametrize("n_past", [7, 300])
def test_attention_projection_fused(libs, consumer, n_past):
    """Decode-token attention block + c_proj (F16) + bias + residual (main-backend.cpp:532-620):
    in tree order one k_attn_proj launch leaves the projection as per-head partial sums; with an
    LN -> F16 GEMV consumer (ln_2 -> c_fc + bias + GELU) the GEMV's prologue adds them and stores
    the residual stream (k_gemv_f16_ps), with any other consumer mi_sum_parts stores it first.
    Both the residual stream and the consumer's output are checked against the reference CPU (tree
    order: within 5e-5 / 2e-4 of max |out|); with the LN consumer the fused graph launches fewer
    kernels than the reference-order one."""
    E, H, F, n_ctx, N = 768, 12, 3072, 1024, 1
    D = E // H
    cur_v = rnd(21, 3 * E, 1.0)
    mem_k, mem_v = rnd(22, E * n_ctx, 1.0), rnd(23, E * n_ctx, 1.0)
    wp = (rnd(24, E * E, 0.05)).astype(np.float16)
    bp, res = rnd(25, E, 0.1), rnd(26, E, 1.0)
    g2, b2 = rnd(27, E, 0.2) + np.float32(1.0), rnd(28, E, 0.1)
    wf = (rnd(29, E * F, 0.05)).astype(np.float16)
    bf = rnd(30, F, 0.1)

    def build(L, c):
        cur = L.ggml_new_tensor_2d(c, F32, 3 * E, N)
        mk, mv = L.ggml_new_tensor_1d(c, F32, E * n_ctx), L.ggml_new_tensor_1d(c, F32, E * n_ctx)
        Wp, Bp, R = L.ggml_new_tensor_2d(c, F16, E, E), L.ggml_new_tensor_1d(c, F32, E), L.ggml_new_tensor_2d(c, F32, E, N)
        G2, B2 = L.ggml_new_tensor_1d(c, F32, E), L.ggml_new_tensor_1d(c, F32, E)
        Wf, Bf = L.ggml_new_tensor_2d(c, F16, E, F), L.ggml_new_tensor_1d(c, F32, F)
        nb1 = cur.contents.nb[1]
        Qcur = L.ggml_view_2d(c, cur, E, N, nb1, 0)
        Kcur = L.ggml_view_2d(c, cur, E, N, nb1, 4 * E)
        Vcur = L.ggml_view_2d(c, cur, E, N, nb1, 8 * E)
        ck = L.ggml_cpy(c, Kcur, L.ggml_view_1d(c, mk, N * E, 4 * E * n_past))
        cv = L.ggml_cpy(c, Vcur, L.ggml_view_1d(c, mv, N * E, 4 * E * n_past))
        Q = L.ggml_permute(c, L.ggml_cont_3d(c, Qcur, D, H, N), 0, 2, 1, 3)
        K = L.ggml_permute(c, L.ggml_reshape_3d(c, L.ggml_view_1d(c, mk, (n_past + N) * E, 0), D, H, n_past + N), 0, 2, 1, 3)
        sm = L.ggml_soft_max(c, L.ggml_diag_mask_inf(c, L.ggml_scale(c, L.ggml_mul_mat(c, K, Q), 1.0 / np.sqrt(D)), n_past))
        Vt = L.ggml_cont_3d(c, L.ggml_permute(c, L.ggml_reshape_3d(c, L.ggml_view_1d(c, mv, (n_past + N) * E, 0), D, H, n_past + N),
                                              1, 2, 0, 3), n_past + N, D, H)
        att = L.ggml_cont_2d(c, L.ggml_permute(c, L.ggml_mul_mat(c, Vt, sm), 0, 2, 1, 3), E, N)
        O = L.ggml_add(c, L.ggml_add(c, L.ggml_mul_mat(c, Wp, att), Bp), R)
        if consumer == "ln_fc":
            h = L.ggml_add(c, L.ggml_mul(c, L.ggml_norm(c, O, 1e-5), G2), B2)
            y = L.ggml_gelu(c, L.ggml_add(c, L.ggml_mul_mat(c, Wf, h), Bf))
        else:
            y = L.ggml_add(c, O, O)
        feeds = [(cur, cur_v), (mk, mem_k), (mv, mem_v), (Wp, wp), (Bp, bp), (R, res), (G2, g2), (B2, b2), (Wf, wf), (Bf, bf)]
        return feeds, [y, O], [ck, cv]

    rt, be, ref, cpu = libs
    (y_a, o_a), n_fast = graph_outputs(rt, be, lambda c: build(rt, c))
    assert rt.ggml_backend_mi355x_set_tuning(b"mmv_order", 1)
    try:
        (y_1, o_1), n_ord = graph_outputs(rt, be, lambda c: build(rt, c))
    finally:
        rt.ggml_backend_mi355x_set_tuning(b"mmv_order", -1)
    (y_r, o_r), _ = graph_outputs(ref, cpu, lambda c: build(ref, c))
    eo = float(np.max(np.abs(o_a - o_r)) / np.max(np.abs(o_r)))
    ey = float(np.max(np.abs(y_a - y_r)) / np.max(np.abs(y_r)))
    print(f"{consumer} n_past={n_past}: residual stream rel err {eo:.2e}, output {ey:.2e}; launches {n_fast} (fused) vs {n_ord}")
    assert eo <= 5e-5 and ey <= 2e-4, (eo, ey)
    # ln_fc: the projection's own GEMV launch is gone; add: it is traded for mi_sum_parts
    assert n_fast < n_ord if consumer == "ln_fc" else n_fast <= n_ord
    # reference order: the unfused kernels, bit for bit
    assert_exact(o_1, o_r, "residual stream, reference order")


# ---- per-node timer (the reference's GGML_PERF, ggml.c:19195-19205) --------------------------------

@pytest.mark.gpu
def test_per_node_timer_fills_perf_fields(capfd):
    """ggml_backend_mi355x_set_perf: every computed node of a graph gets perf_runs per compute and
    device microseconds (a fused chain's time on its last node); the node times add up to at most
    the graph's; ggml_graph_print prints the reference's table."""
    import ctypes
    lib = G.runtime()
    be = G.mi355x_backend(lib)
    try:
        lib.ggml_backend_mi355x_set_perf(be, True)
        K, N, B = 4096, 4096, 4
        overhead = lib.ggml_tensor_overhead() * 16 + lib.ggml_graph_overhead()
        with G.Context(lib, overhead, no_alloc=True) as c:
            w = lib.ggml_new_tensor_2d(c.ctx, G.GGML_TYPE_F16, K, N)
            x = lib.ggml_new_tensor_2d(c.ctx, G.GGML_TYPE_F32, K, B)
            y = lib.ggml_mul_mat(c.ctx, w, x)
            z = lib.ggml_scale(c.ctx, y, 0.5)
            out = lib.ggml_soft_max(c.ctx, z)
            g = lib.ggml_new_graph(c.ctx)
            lib.ggml_build_forward_expand(g, out)
            buf = lib.ggml_backend_alloc_ctx_tensors(c.ctx, be)
            try:
                G.tensor_set(lib, w, (np.random.default_rng(1).standard_normal(K * N) * 0.01).astype(np.float16))
                G.tensor_set(lib, x, np.random.default_rng(2).standard_normal(K * B).astype(np.float32))
                for _ in range(3):
                    assert lib.ggml_backend_graph_compute(be, g) == G.GGML_STATUS_SUCCESS
                gc = g.contents
                nodes = [gc.nodes[i].contents for i in range(gc.n_nodes)]
                assert all(n.perf_runs == 3 for n in nodes), [n.perf_runs for n in nodes]
                mm = [n for n in nodes if n.op == G.GGML_OP_MUL_MAT][0]
                assert mm.perf_time_us > 0
                assert gc.perf_runs == 3
                assert sum(n.perf_time_us for n in nodes) <= gc.perf_time_us + len(nodes)
                lib.ggml_graph_print(g)
            finally:
                lib.ggml_backend_buffer_free(buf)
        printed = capfd.readouterr().out
        assert "=== GRAPH ===" in printed and "MUL_MAT" in printed and "perf_total_per_op_us" in printed
    finally:
        lib.ggml_backend_mi355x_set_perf(be, False)
        lib.ggml_backend_free(be)


@pytest.mark.parametrize("bn", [0, 1, 3, 5])
@pytest.mark.parametrize("K,N,ncols,epi", [(768, 2304, 8, "bias"), (768, 3072, 5, "gelu"), (512, 200, 2, "none"), (1024, 96, 3, "bias")])
def test_norm_prologue_gemv_columns(libs, bn, K, N, ncols, epi):
    """norm -> mul(g) -> add(b) -> F16 mul_mat (+ bias, + GELU) of 2..8 columns, the batched-decode
    shape of GPT-2's c_attn / c_fc (main-batched.cpp): in tree order one launch whose prologue
    normalizes the columns (f16_bn 1-5: k_gemv_f16_bn, every column normalized once per workgroup,
    4 / 8 / 16 waves, K split over 1 / 2 / 4 waves; 0: the earlier k_gemv_f16 forms) -- within the
    F16 decode tolerance (1e-3 rel) of the reference CPU, and the shapes agree with each other."""
    rt = libs[0]
    x = rnd(40 + K, K * ncols, 2.0)
    g = rnd(41, K, 1.0) + np.float32(1.0)
    bb = rnd(42, K, 0.1)
    w = (rnd(43, K * N, 0.05)).astype(np.float16)
    bias = rnd(44, N, 0.2)

    def build(L, c):
        t = L.ggml_new_tensor_2d(c, F32, K, ncols)
        gt = L.ggml_new_tensor_1d(c, F32, K)
        bt = L.ggml_new_tensor_1d(c, F32, K)
        wt = L.ggml_new_tensor_2d(c, F16, K, N)
        bi = L.ggml_new_tensor_1d(c, F32, N)
        h = L.ggml_add(c, L.ggml_mul(c, L.ggml_norm(c, t, 1e-5), gt), bt)
        y = L.ggml_mul_mat(c, wt, h)
        if epi != "none":
            y = L.ggml_add(c, y, bi)
        if epi == "gelu":
            y = L.ggml_gelu(c, y)
        return [(t, x), (gt, g), (bt, bb), (wt, w), (bi, bias)], y

    try:
        assert rt.ggml_backend_mi355x_set_tuning(b"f16_bn", bn)
        assert rt.ggml_backend_mi355x_set_tuning(b"mmv_order", 0)
        a, b = both(libs, build)
    finally:
        rt.ggml_backend_mi355x_set_tuning(b"f16_bn", 5)
        rt.ggml_backend_mi355x_set_tuning(b"mmv_order", -1)
    rel = float(np.abs(a.astype(np.float64) - b).max() / np.abs(b).max())
    print(f"f16_bn={bn} K={K} N={N} cols={ncols} {epi}: max rel {rel:.2e}")
    assert rel <= 1e-3


@pytest.mark.parametrize("bp", [0, 1])
@pytest.mark.parametrize("K,N,ncols,epi", [(768, 768, 8, "resid"), (3072, 768, 8, "resid"), (1000, 130, 3, "bias"), (256, 64, 2, "none")])
def test_plain_gemv_columns(libs, bp, K, N, ncols, epi):
    """F16 mul_mat of 2..8 plain columns (+ bias, + residual): batched decode's c_proj / mlp projection.
    f16_bp 1: 16-wave workgroups of 16 rows, K split over 4 waves, the columns staged once per
    workgroup (k_gemv_f16_bn's plain form; measured slower on batched decode, 0.63-0.64 vs 0.59-0.60
    ms/step, profiles/r06r_batched_plain_gemv_ab.txt: diagnostic builds only); 0: k_gemv_f16. Within
    1e-3 rel of the reference CPU."""
    rt = libs[0]
    x = rnd(50 + K, K * ncols, 1.0)
    w = (rnd(51, K * N, 0.05)).astype(np.float16)
    bias = rnd(52, N, 0.2)
    res = rnd(53, N * ncols, 1.0)

    def build(L, c):
        t = L.ggml_new_tensor_2d(c, F32, K, ncols)
        wt = L.ggml_new_tensor_2d(c, F16, K, N)
        bi = L.ggml_new_tensor_1d(c, F32, N)
        rs = L.ggml_new_tensor_2d(c, F32, N, ncols)
        y = L.ggml_mul_mat(c, wt, t)
        if epi != "none":
            y = L.ggml_add(c, y, bi)
        if epi == "resid":
            y = L.ggml_add(c, y, rs)
        return [(t, x), (wt, w), (bi, bias), (rs, res)], y

    try:
        if not rt.ggml_backend_mi355x_set_tuning(b"f16_bp", bp):
            pytest.skip("f16_bp 1: diagnostic builds only (measured slower)")
        assert rt.ggml_backend_mi355x_set_tuning(b"mmv_order", 0)
        a, b = both(libs, build)
    finally:
        rt.ggml_backend_mi355x_set_tuning(b"f16_bp", 0)
        rt.ggml_backend_mi355x_set_tuning(b"mmv_order", -1)
    rel = float(np.abs(a.astype(np.float64) - b).max() / np.abs(b).max())
    assert rel <= 1e-3, rel
