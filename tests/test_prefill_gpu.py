"""Batched (prompt / prefill) GGML_OP_MUL_MAT at BASELINE sizes: configs[4] (Q4_K 4096x4096,
B=512, prompt-sharded over GPUs) and the mid-batch sizes B in {9, 16, 32, 64}.

The reference outputs are the P_* golden cases (tests/golden/make_golden.py, written by the
reference CPU mul_mat, ggml.c:11808-12097 -> vec_dot_q4_K_q8_K, ggml-quants.c:7089-7152): the
SHA-256 of the whole Y plus every step-th column. Three checks:
  * the sampled columns, element-wise, within 1e-5 of max|y| (the prefill GEMM computes the
    reference's exact integer block sums; only the f32 combine order differs);
  * the WHOLE Y at full size: the decode GEMV in mmv_order=1 is bit-identical to the reference
    CPU (test_mul_mat_gpu.py), so its 8-column slices reassemble the reference Y -- its SHA-256
    must equal the fixture's -- and every element of the prefill Y is checked against it;
  * prompt sharding (configs[4] on 8 GPUs, 64 columns each): the column shards computed alone
    concatenate to the unsharded result bit for bit.
"""
import ctypes
import hashlib

import numpy as np
import pytest

from conftest import golden_blob, golden_cases
import pyoracle as orc
from ggml_mi355x import ggml as G
from ggml_mi355x import synth

pytestmark = pytest.mark.gpu

PREFILL = golden_cases(large=True, prefill=True)
EXACT_TOL = 1e-5


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


def _inputs(rt, c):
    K, N, B = c["K"], c["N"], c["B"]
    w = synth.uniform(c["wseed"], K * N)
    wq = np.empty(c["wq_bytes"], np.uint8)
    rt.ggml_quantize_chunk(c["type"], w.ctypes.data, wq.ctypes.data, 0, N, K, None)
    assert hashlib.sha256(wq.tobytes()).hexdigest() == c["wq_sha256"], "runtime quantizer != reference bytes"
    return wq, synth.uniform(c["xseed"], K * B)


def _reference_y_by_gemv(rt, backend, t, wq, K, N, x, B):
    """Y [B, N] from the bit-exact decode path (mmv_order=1), 8 columns per mul_mat."""
    assert rt.ggml_backend_mi355x_set_tuning(b"mmv_order", 1)
    try:
        xs = x.reshape(B, K)
        cols = [G.mul_mat_once(rt, backend, t, wq, K, N, np.ascontiguousarray(xs[c0:c0 + 8]).ravel(), min(8, B - c0))
                for c0 in range(0, B, 8)]
    finally:
        rt.ggml_backend_mi355x_set_tuning(b"mmv_order", -1)
    return np.concatenate(cols).reshape(B, N)


@pytest.mark.parametrize("c", PREFILL, ids=[c["name"] for c in PREFILL])
def test_prefill_matches_reference_at_full_size(rt, backend, c):
    K, N, B, t = c["K"], c["N"], c["B"], c["type"]
    wq, x = _inputs(rt, c)
    y = G.mul_mat_once(rt, backend, t, wq, K, N, x, B).reshape(B, N)
    step = c["y_col_step"]
    ys = golden_blob(c["name"] + ".ys.f32", np.float32).reshape(-1, N)
    err_s = rel_err(y[::step], ys)
    yref = _reference_y_by_gemv(rt, backend, t, wq, K, N, x, B)
    assert hashlib.sha256(yref.tobytes()).hexdigest() == c["y_sha256"], "GEMV reassembly != reference Y"
    err = rel_err(y, yref)
    same = float(np.mean(y.view(np.uint32) == yref.view(np.uint32)))
    print(f"{c['name']}: sampled columns {err_s:.2e}, whole Y {err:.2e}, bit-identical elements {same:.3f}")
    assert err_s <= EXACT_TOL, err_s
    assert err <= EXACT_TOL, err


@pytest.mark.parametrize("world", [8, 3])
def test_prompt_sharded_prefill_equals_whole(rt, backend, world):
    """configs[4] prompt sharding: shard_range(512, world, r) columns per rank, each computed alone
    (as each GPU does), concatenate to the whole B=512 product bit for bit."""
    import bench
    c = next(cc for cc in PREFILL if cc["B"] == 512)
    K, N, B, t = c["K"], c["N"], c["B"], c["type"]
    wq, x = _inputs(rt, c)
    whole = G.mul_mat_once(rt, backend, t, wq, K, N, x, B).reshape(B, N)
    xs = x.reshape(B, K)
    parts = []
    for r in range(world):
        s0, cnt = bench.shard_range(B, world, r)
        parts.append(G.mul_mat_once(rt, backend, t, wq, K, N, np.ascontiguousarray(xs[s0:s0 + cnt]).ravel(), cnt).reshape(cnt, N))
    sharded = np.concatenate(parts)
    assert np.array_equal(sharded.view(np.uint32), whole.view(np.uint32)), rel_err(sharded, whole)


@pytest.mark.parametrize("tname", ["q4_K", "q5_K", "q4_0", "q8_0"])
@pytest.mark.parametrize("K,N,B", [(256, 64, 9), (512, 100, 130), (768, 2304, 24), (3072, 768, 40), (1280, 96, 257)])
def test_prefill_exact_gemm_shapes_vs_oracle(rt, backend, tname, K, N, B):
    """Ragged tiles (N, B not multiples of 64 / 128), odd superblock counts (the canonical chain
    split puts the extra superblock in the second half), one-superblock rows. Q4_0 / Q8_0 run the
    same exact-integer scheme on k_mmq0p (one i8 MFMA per 32-block, q8_0 activations)."""
    t = orc.TYPES_BY_NAME[tname]
    w = synth.uniform(K * 7 + N, K * N)
    x = synth.uniform(K * 3 + B, K * B)
    wq = orc.quantize(t, w, K)
    y = G.mul_mat_once(rt, backend, t, wq, K, N, x, B)
    ref = orc.mul_mat(t, wq, K, N, x, B)
    err = rel_err(y, ref)
    print(f"{tname} {K}x{N}x{B}: {err:.2e}")
    assert err <= EXACT_TOL, err


def test_prefill_edge_values(rt, backend):
    """All-zero activation superblocks (d = 0), constant weight rows (d_w = 0, mins only) and
    saturated quants: the exact-integer path against the oracle."""
    t, K, N, B = orc.Q4_K, 1024, 96, 40
    w = synth.uniform(5, K * N).reshape(N, K)
    w[3] = 0.25          # constant rows: every sub-block scale 0, mins carry the value
    w[7] = 0.0
    w[11, :256] = 1.0    # one constant superblock
    x = synth.uniform(6, K * B).reshape(B, K)
    x[2] = 0.0           # all-zero columns / superblocks
    x[5, 256:512] = 0.0
    x[9] = np.where(np.arange(K) % 2, 1e3, -1e3)  # saturated quants
    wq = orc.quantize(t, np.ascontiguousarray(w).ravel(), K)
    y = G.mul_mat_once(rt, backend, t, wq, K, N, np.ascontiguousarray(x).ravel(), B)
    ref = orc.mul_mat(t, wq, K, N, np.ascontiguousarray(x).ravel(), B)
    assert np.all(np.isfinite(y))
    assert rel_err(y, ref) <= EXACT_TOL


@pytest.mark.parametrize("tname", ["q4_K", "q5_K", "q4_0", "q8_0"])
@pytest.mark.parametrize("B", [72, 13])
def test_prefill_kernels_bit_equal(rt, backend, tname, B):
    """Every prefill kernel shares the canonical combine (exact T and U per superblock, terms
    combined in the cfold order: 8 contiguous superblock groups, each left-folded; groups 0-3 and
    4-7 left-folded separately, then added), so any kernel choice gives the same bits: k_mmqp (the default for <= 128
    columns), k_mmqd1 (variant bit 2048), k_mmqx (full- and half-width workgroups) and, for <= 16
    columns, k_mmqd16 (variant bit 2^21; 16 x 16 tiles on the 16x16x64 MFMA). Q4_0 / Q8_0:
    k_mmq0p (32 x 32 tiles, <= 64 columns) and k_mmq0x (weights staged per 64 x 128 workgroup)."""
    t = orc.TYPES_BY_NAME[tname]
    K, N = 4096, 320
    w = synth.uniform(11, K * N)
    x = synth.uniform(12, K * B)
    wq = orc.quantize(t, w, K)
    if tname in ("q4_0", "q8_0"):  # k_mmq0p (16), k_mmq0x full / half width (128, 128 | 65536)
        variants = [0, 16, 128, 128 | 65536, 128 | (1 << 24), 128 | (1 << 25)]
    else:
        variants = [0, 2048, 1 << 27, 128 | 131072, 128 | 65536, 128 | 131072 | (1 << 28)] + ([1 << 21] if B <= 16 else [])
    # long-prompt kernels forced onto these shapes (variant bits 128 | 131072, mmq_long): k_mmqw (1,
    # diagnostic builds only for Q4_K), k_mmqt (2, K split over wave pairs, Q4_K)
    longs = [(128 | 131072, L) for L in (1, 2)] if tname in ("q4_K", "q5_K") else []
    if longs and not rt.ggml_backend_mi355x_set_tuning(b"mmq_long", 1):
        longs = longs[1:]
    outs = {}
    try:
        for v in variants + longs:
            vv, lng = v if isinstance(v, tuple) else (v, 0)
            assert rt.ggml_backend_mi355x_set_tuning(b"mmq_variant", vv)
            assert rt.ggml_backend_mi355x_set_tuning(b"mmq_long", lng)
            outs[v] = G.mul_mat_once(rt, backend, t, wq, K, N, x, B)
    finally:
        rt.ggml_backend_mi355x_set_tuning(b"mmq_variant", 0)
        rt.ggml_backend_mi355x_set_tuning(b"mmq_long", 0)
    variants = variants + longs
    ref = orc.mul_mat(t, wq, K, N, x, B)
    assert rel_err(outs[0], ref) <= EXACT_TOL
    for v in variants[1:]:
        assert np.array_equal(outs[v].view(np.uint32), outs[0].view(np.uint32)), (v, rel_err(outs[v], outs[0]))


@pytest.mark.parametrize("lng", [2, 3, 4, 5])
@pytest.mark.parametrize("K,N,B", [(256, 64, 130), (1280, 96, 257), (3072, 200, 200), (11008, 256, 136), (4096, 4096, 512)])
def test_split_k_prefill_bit_equal(rt, backend, K, N, B, lng):
    """k_mmqt (mmq_long 2, the Q4_K kernel past 128 columns without repacked planes: the two K
    halves of the canonical order on two waves, met in LDS; diagnostic builds also mmq_long 5, the
    same with the high half's combine deferred one stage (staggered), mmq_long 3, the
    same with each half's stages synchronized on its own, and 4, k_mmqv: one wave per SIMD over the
    whole K with the combine software-pipelined under the next superblock's MFMAs) forced onto
    ragged shapes: one superblock (empty high half), S = 5 (a one-superblock high half), S = 12,
    S = 43 (a high half shorter than the low: idle steps), ragged rows and columns; bit-identical to
    the default kernel (k_mmqr on the planes) and within the exact-path tolerance of the oracle."""
    t = orc.Q4_K
    w = synth.uniform(K + 3 * N, K * N)
    x = synth.uniform(K + 5 * B, K * B)
    wq = orc.quantize(t, w, K)
    try:
        base = G.mul_mat_once(rt, backend, t, wq, K, N, x, B)
        assert rt.ggml_backend_mi355x_set_tuning(b"mmq_variant", 128 | 131072)
        if not rt.ggml_backend_mi355x_set_tuning(b"mmq_long", lng):
            pytest.skip("mmq_long %d: diagnostic builds only (measured slower)" % lng)
        y = G.mul_mat_once(rt, backend, t, wq, K, N, x, B)
    finally:
        rt.ggml_backend_mi355x_set_tuning(b"mmq_variant", 0)
        rt.ggml_backend_mi355x_set_tuning(b"mmq_long", 0)
    assert np.array_equal(y.view(np.uint32), base.view(np.uint32)), rel_err(y, base)
    if K * N * B <= 4096 * 4096 * 64:
        assert rel_err(y, orc.mul_mat(t, wq, K, N, x, B)) <= EXACT_TOL


@pytest.mark.parametrize("tname", ["q4_K", "q5_K", "q4_0", "q8_0"])
@pytest.mark.parametrize("B", [64, 13, 300])
def test_grouped_prefill_equals_single(rt, backend, tname, B):
    """Independent batched mul_mats of one graph (five members: two share one src1, weights of
    different row counts) run as one quantizer launch + one grouped GEMM launch; every member's
    output is bit-identical to the same mul_mat computed alone."""
    t = orc.TYPES_BY_NAME[tname]
    K = 2048
    Ns = [512, 320, 512, 96, 1024]
    srcs = [0, 1, 1, 2, 3]  # member -> activation source
    ovh = rt.ggml_tensor_overhead() * 24 + rt.ggml_graph_overhead()
    ctx = G.Context(rt, ovh, no_alloc=True)
    c = ctx.ctx
    ws = [rt.ggml_new_tensor_2d(c, t, K, n) for n in Ns]
    xs = [rt.ggml_new_tensor_2d(c, G.GGML_TYPE_F32, K, B) for _ in range(4)]
    ys = [rt.ggml_mul_mat(c, w, xs[s]) for w, s in zip(ws, srcs)]
    g = rt.ggml_new_graph(c)
    for y in ys:
        rt.ggml_build_forward_expand(g, y)
    buf = rt.ggml_backend_alloc_ctx_tensors(c, backend)
    try:
        wqs = [orc.quantize(t, synth.uniform(30 + i, K * n), K) for i, n in enumerate(Ns)]
        xv = [synth.uniform(40 + i, K * B) for i in range(4)]
        for w, wq in zip(ws, wqs):
            G.tensor_set(rt, w, wq)
        for x, v in zip(xs, xv):
            G.tensor_set(rt, x, v)
        assert rt.ggml_backend_graph_compute(backend, g) == G.GGML_STATUS_SUCCESS
        assert rt.ggml_backend_mi355x_last_launch_count(backend) == 2
        for i, (y, n, s) in enumerate(zip(ys, Ns, srcs)):
            got = G.tensor_get(rt, y)
            alone = G.mul_mat_once(rt, backend, t, wqs[i], K, n, xv[s], B)
            assert np.array_equal(got.view(np.uint32), alone.view(np.uint32)), (i, rel_err(got, alone))
        ref = orc.mul_mat(t, wqs[4], K, Ns[4], xv[3], B)
        assert rel_err(G.tensor_get(rt, ys[4]), ref) <= EXACT_TOL
    finally:
        rt.ggml_backend_buffer_free(buf)
        ctx.free()


@pytest.mark.parametrize("tname", ["q5_K", "q4_K"])
def test_long_prefill_into_host_memory(rt, backend, tname):
    """A long prompt (> 128 columns, where k_mmqw / k_mmqx keep a partial sum in their own output
    locations until the end) whose output lives in pinned host memory (the host buffer type, e.g.
    host-staged logits): the backend picks a kernel that stores each output once; the result is
    bit-identical to the same mul_mat into device memory."""
    t = orc.TYPES_BY_NAME[tname]
    K, N, B = 2048, 320, 160
    wq = orc.quantize(t, synth.uniform(71, K * N), K)
    x = synth.uniform(72, K * B)
    dev_y = G.mul_mat_once(rt, backend, t, wq, K, N, x, B)
    ovh = rt.ggml_tensor_overhead() * 8 + rt.ggml_graph_overhead()
    cd, ch = G.Context(rt, ovh, no_alloc=True), G.Context(rt, ovh, no_alloc=True)
    try:
        w = rt.ggml_new_tensor_2d(cd.ctx, t, K, N)
        xt = rt.ggml_new_tensor_2d(cd.ctx, G.GGML_TYPE_F32, K, B)
        y = rt.ggml_mul_mat(ch.ctx, w, xt)  # the result tensor belongs to the host-buffer context
        g = rt.ggml_new_graph(ch.ctx)
        rt.ggml_build_forward_expand(g, y)
        bd = rt.ggml_backend_alloc_ctx_tensors(cd.ctx, backend)
        bh = rt.ggml_backend_alloc_ctx_tensors_from_buft(ch.ctx, rt.ggml_backend_mi355x_host_buffer_type())
        assert bd and bh
        try:
            assert rt.ggml_backend_buffer_is_host(bh)
            G.tensor_set(rt, w, wq)
            G.tensor_set(rt, xt, x)
            assert rt.ggml_backend_graph_compute(backend, g) == G.GGML_STATUS_SUCCESS
            host_y = G.tensor_get(rt, y)
        finally:
            rt.ggml_backend_buffer_free(bh)
            rt.ggml_backend_buffer_free(bd)
    finally:
        ch.free()
        cd.free()
    assert np.array_equal(host_y.view(np.uint32), dev_y.view(np.uint32)), rel_err(host_y, dev_y)
    assert rel_err(dev_y, orc.mul_mat(t, wq, K, N, x, B)) <= EXACT_TOL


def _planes_stats(rt):
    b = ctypes.c_size_t(0)
    n = rt.ggml_backend_mi355x_planes_stats(ctypes.byref(b))
    return int(n), int(b.value)


@pytest.mark.parametrize("tname,K,N,B", [("q4_K", 256, 64, 130), ("q4_K", 1280, 96, 257), ("q4_K", 3072, 200, 200),
                                         ("q4_K", 11008, 256, 136), ("q4_K", 4096, 4096, 512), ("q5_K", 1280, 96, 257),
                                         ("q5_K", 4096, 1024, 512), ("q5_K", 2816, 130, 129)])
def test_planes_prefill_bit_equal_canonical(rt, backend, tname, K, N, B):
    """Long prompts (> 128 columns) on the repacked MFMA planes (mmq_planes.hip k_mmqr; Q4_K -- Q5_K
    keeps the canonical kernels, the case checks the switch) against the
    canonical kernels on the raw blocks (planes off: k_mmqt / k_mmqw): the same exact integer sums
    and the same cfold combine, so bit-identical -- ragged rows (N % 64, N % 32), ragged columns,
    one superblock (empty high half), odd superblock counts; and within the exact-path tolerance
    of the oracle."""
    t = orc.TYPES_BY_NAME[tname]
    w = synth.uniform(K + 11 * N, K * N)
    x = synth.uniform(K + 13 * B, K * B)
    wq = orc.quantize(t, w, K)
    base = G.mul_mat_once(rt, backend, t, wq, K, N, x, B)  # (planes are opt-in: off by default)
    n0, _ = _planes_stats(rt)
    try:
        assert rt.ggml_backend_mi355x_set_tuning(b"planes", 1)
        y = G.mul_mat_once(rt, backend, t, wq, K, N, x, B)
    finally:
        rt.ggml_backend_mi355x_set_tuning(b"planes", 0)
    assert _planes_stats(rt)[0] == n0, "planes of a freed buffer must be dropped with it"
    assert np.array_equal(y.view(np.uint32), base.view(np.uint32)), rel_err(y, base)
    if K * N * B <= 4096 * 1024 * 64:
        assert rel_err(y, orc.mul_mat(t, wq, K, N, x, B)) <= EXACT_TOL


@pytest.mark.parametrize("tname", ["q4_K"])
def test_planes_follow_weight_writes(rt, backend, tname):
    """The planes are a device-side copy next to the canonical blocks: set_tensor -> get_tensor
    round-trips the reference bytes exactly (also after partial-offset writes), and a partial
    rewrite of some rows (offset into the tensor) renews the planes, so the next long prompt sees
    the new weights (compared with the oracle and with the canonical kernels)."""
    t = orc.TYPES_BY_NAME[tname]
    K, N, B = 2048, 192, 160
    rb = orc.row_size(t, K)
    wq = orc.quantize(t, synth.uniform(81, K * N), K)
    wq2 = orc.quantize(t, synth.uniform(82, K * N), K)
    x = synth.uniform(83, K * B)
    ovh = rt.ggml_tensor_overhead() * 8 + rt.ggml_graph_overhead()
    with G.Context(rt, ovh, no_alloc=True) as c:
        w = rt.ggml_new_tensor_2d(c.ctx, t, K, N)
        xt = rt.ggml_new_tensor_2d(c.ctx, G.GGML_TYPE_F32, K, B)
        y = rt.ggml_mul_mat(c.ctx, w, xt)
        g = rt.ggml_new_graph(c.ctx)
        rt.ggml_build_forward_expand(g, y)
        buf = rt.ggml_backend_alloc_ctx_tensors(c.ctx, backend)
        assert buf
        assert rt.ggml_backend_mi355x_set_tuning(b"planes", 1)
        try:
            n0, _ = _planes_stats(rt)
            G.tensor_set(rt, w, wq)
            G.tensor_set(rt, xt, x)
            assert rt.ggml_backend_graph_compute(backend, g) == G.GGML_STATUS_SUCCESS
            n1, nbytes = _planes_stats(rt)
            assert n1 == n0 + 1 and nbytes > 0, "the long prompt did not create the weight's planes"
            y1 = G.tensor_get(rt, y)
            assert rel_err(y1, orc.mul_mat(t, wq, K, N, x, B)) <= EXACT_TOL
            back = np.empty_like(wq)
            rt.ggml_backend_tensor_get(w, back.ctypes.data, 0, back.nbytes)
            assert np.array_equal(back, wq), "get_tensor must return the canonical bytes"
            # rows 37 .. 120 replaced, at an offset into the tensor (not row-tile aligned)
            mixed = wq.copy()
            lo, hi = 37 * rb, 121 * rb
            mixed[lo:hi] = wq2[lo:hi]
            G.tensor_set(rt, w, wq2[lo:hi], offset=lo)
            rt.ggml_backend_tensor_get(w, back.ctypes.data, 0, back.nbytes)
            assert np.array_equal(back, mixed)
            assert rt.ggml_backend_graph_compute(backend, g) == G.GGML_STATUS_SUCCESS
            y2 = G.tensor_get(rt, y)
            assert rel_err(y2, orc.mul_mat(t, mixed, K, N, x, B)) <= EXACT_TOL
            # an ASYNC write on the backend's stream (ggml_backend_tensor_set_async) renews them too
            mixed_a = mixed.copy()
            lo2, hi2 = 150 * rb, 170 * rb
            chunk = np.ascontiguousarray(wq[lo2:hi2])
            mixed_a[lo2:hi2] = chunk
            rt.ggml_backend_tensor_set_async(backend, w, chunk.ctypes.data, lo2, chunk.nbytes)
            assert rt.ggml_backend_graph_compute(backend, g) == G.GGML_STATUS_SUCCESS
            rt.ggml_backend_synchronize(backend)
            y2a = G.tensor_get(rt, y)
            assert rel_err(y2a, orc.mul_mat(t, mixed_a, K, N, x, B)) <= EXACT_TOL
            mixed = mixed_a
            y2 = y2a
            assert rt.ggml_backend_mi355x_set_tuning(b"planes", 0)
            assert rt.ggml_backend_graph_compute(backend, g) == G.GGML_STATUS_SUCCESS
            y3 = G.tensor_get(rt, y)
            assert np.array_equal(y2.view(np.uint32), y3.view(np.uint32)), rel_err(y2, y3)
        finally:
            rt.ggml_backend_mi355x_set_tuning(b"planes", 0)
            rt.ggml_backend_buffer_free(buf)
    assert _planes_stats(rt)[0] == n0


def _graph_stats(rt, be):
    arr = (ctypes.c_int64 * 6)()
    assert rt.ggml_backend_mi355x_graph_stats_ex(be, arr, 6) == 6
    return list(arr)


def test_planes_captured_graph_after_weight_realloc(rt, backend):
    """Captured graphs bake in the repacked planes' address (mi_mmx_member::planes): a weight buffer
    freed and a new one allocated -- usually at the same address, same shapes, so every tensor
    address of the graph key repeats -- must not replay a capture that reads the freed planes
    (the planes generation is part of the graph key). Two long-prompt mul_mats in a chain (4
    launches: captured on the second compute, replayed on the third), each round with new weights,
    bit-identical to the canonical kernels (planes off) on the same inputs."""
    t = orc.Q4_K
    K = N = 1024
    B = 160
    x = synth.uniform(91, K * B)

    def run(wq, planes, reps):
        ovh = rt.ggml_tensor_overhead() * 8 + rt.ggml_graph_overhead()
        with G.Context(rt, ovh, no_alloc=True) as cw, G.Context(rt, ovh, no_alloc=True) as cc:
            w = rt.ggml_new_tensor_2d(cw.ctx, t, K, N)
            bw = rt.ggml_backend_alloc_ctx_tensors(cw.ctx, backend)
            xt = rt.ggml_new_tensor_2d(cc.ctx, G.GGML_TYPE_F32, K, B)
            y2 = rt.ggml_mul_mat(cc.ctx, w, rt.ggml_mul_mat(cc.ctx, w, xt))
            g = rt.ggml_new_graph(cc.ctx)
            rt.ggml_build_forward_expand(g, y2)
            bc = rt.ggml_backend_alloc_ctx_tensors(cc.ctx, backend)
            assert bw and bc
            addr = rt.ggml_backend_buffer_get_base(bw)
            try:
                assert rt.ggml_backend_mi355x_set_tuning(b"planes", planes)
                # (the chain's second mul_mat consumes a computed value: the per-graph order would pick
                # the reference-order prompt path; the tree order keeps the MFMA GEMMs on the planes)
                assert rt.ggml_backend_mi355x_set_tuning(b"mmv_order", 0)
                G.tensor_set(rt, w, wq)
                G.tensor_set(rt, xt, x)
                outs = []
                for _ in range(reps):
                    assert rt.ggml_backend_graph_compute(backend, g) == G.GGML_STATUS_SUCCESS
                    outs.append(G.tensor_get(rt, y2))
            finally:
                rt.ggml_backend_mi355x_set_tuning(b"planes", 0)
                rt.ggml_backend_mi355x_set_tuning(b"mmv_order", -1)
                rt.ggml_backend_buffer_free(bc)
                rt.ggml_backend_buffer_free(bw)
            return outs, addr

    n0, _ = _planes_stats(rt)
    for seed in (92, 93):
        wq = orc.quantize(t, synth.uniform(seed, K * N), K)
        base, _ = run(wq, 0, 1)
        s0 = _graph_stats(rt, backend)
        outs, _ = run(wq, 1, 3)
        s1 = _graph_stats(rt, backend)
        assert s1[4] > s0[4], "the chain was never replayed from a capture: the case tests nothing"
        for y in outs:
            assert np.array_equal(y.view(np.uint32), base[0].view(np.uint32)), rel_err(y, base[0])
    assert _planes_stats(rt)[0] == n0


@pytest.mark.parametrize("B", [33, 64, 100, 128])
def test_short_prompt_mmqt_route_bit_equal(rt, backend, B):
    """Q4_K prompts of 33..128 columns take k_mmqt (128 x 64 tiles) when the launch has at least
    mmqt_short of its workgroups (default 192: grouped launches that nearly fill the chip), else k_mmqp.
    Forced on (mmqt_short 1) over ragged rows and columns, it is bit-identical to k_mmqp (off)
    and within the exact-path tolerance of the oracle."""
    t = orc.Q4_K
    K = 2048
    Ns = [512, 320, 96, 1024]
    wqs = [orc.quantize(t, synth.uniform(60 + i, K * n), K) for i, n in enumerate(Ns)]
    xs = [synth.uniform(70 + i, K * B) for i in range(len(Ns))]

    def run(mmqt_short):
        ovh = rt.ggml_tensor_overhead() * 24 + rt.ggml_graph_overhead()
        with G.Context(rt, ovh, no_alloc=True) as c:
            ws = [rt.ggml_new_tensor_2d(c.ctx, t, K, n) for n in Ns]
            xts = [rt.ggml_new_tensor_2d(c.ctx, G.GGML_TYPE_F32, K, B) for _ in Ns]
            ys = [rt.ggml_mul_mat(c.ctx, w, x) for w, x in zip(ws, xts)]
            g = rt.ggml_new_graph(c.ctx)
            for y in ys:
                rt.ggml_build_forward_expand(g, y)
            buf = rt.ggml_backend_alloc_ctx_tensors(c.ctx, backend)
            assert buf
            try:
                assert rt.ggml_backend_mi355x_set_tuning(b"mmqt_short", mmqt_short)
                for w, wq, x, xv in zip(ws, wqs, xts, xs):
                    G.tensor_set(rt, w, wq)
                    G.tensor_set(rt, x, xv)
                assert rt.ggml_backend_graph_compute(backend, g) == G.GGML_STATUS_SUCCESS
                assert rt.ggml_backend_mi355x_last_launch_count(backend) == 2  # one quantizer + one grouped GEMM
                return [G.tensor_get(rt, y) for y in ys]
            finally:
                rt.ggml_backend_mi355x_set_tuning(b"mmqt_short", 192)
                rt.ggml_backend_buffer_free(buf)

    forced, base = run(1), run(0)
    for i in range(len(Ns)):
        assert np.array_equal(forced[i].view(np.uint32), base[i].view(np.uint32)), (i, rel_err(forced[i], base[i]))
    assert rel_err(forced[1], orc.mul_mat(t, wqs[1], K, Ns[1], xs[1], B)) <= EXACT_TOL
