"""CPU tests of the runtime's host side (no GPU): ABI, exports, type table, fp16, quantizers,
graph construction and allocation -- checked against the reference libggml where it is built
(oracle/_ref, this container) and against the golden vectors everywhere."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import REPO, golden_blob, golden_cases
from ggml_mi355x import ggml as G
from ggml_mi355x import synth

REF_LIB = os.path.join(REPO, "oracle", "_ref", "libggml_ref.so")
needs_ref = pytest.mark.skipif(not os.path.exists(REF_LIB), reason="reference build (oracle/_ref) absent")


@pytest.fixture(scope="module")
def rt():
    return G.runtime()


@pytest.fixture(scope="module")
def ref():
    return G.Lib([REF_LIB], isolated=True)


def _declared(header):
    txt = open(os.path.join(REPO, "include", header)).read()
    return sorted(set(re.findall(r"GGML_API\s+[^;(]*?\b(ggml_\w+)\s*\(", txt)))


def test_backend_exports_every_declared_symbol(rt):
    lib = ctypes.CDLL(G.BACKEND_LIB)
    names = _declared("ggml-mi355x.h")
    assert len(names) >= 14
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_core_exports_every_declared_symbol(rt):
    lib = ctypes.CDLL(G.CORE_LIB)
    names = _declared("ggml_abi.h")
    assert len(names) > 100
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_backend_plugin_needs_only_core_api():
    """The backend's undefined ggml symbols must all exist in the reference libggml too, so it
    loads into the reference unchanged (the drop-in claim)."""
    import subprocess
    out = subprocess.check_output(["nm", "-D", "--undefined-only", G.BACKEND_LIB], text=True)
    und = sorted({l.split()[-1] for l in out.splitlines() if l.split()[-1].startswith("ggml_")})
    assert und, "expected references into the ggml API"
    core = ctypes.CDLL(G.CORE_LIB)
    assert all(hasattr(core, n) for n in und)
    if os.path.exists(REF_LIB):
        reflib = G.Lib([REF_LIB], isolated=True).handles[0]
        assert all(hasattr(reflib, n) for n in und), [n for n in und if not hasattr(reflib, n)]


def test_no_devices_without_gpu(rt):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    assert rt.ggml_backend_mi355x_get_device_count() == 0
    assert rt.ggml_backend_reg_get_count() == 0


@needs_ref
def test_type_table_matches_reference(rt, ref):
    for t in list(range(0, 4)) + list(range(6, 31)):
        assert rt.ggml_type_size(t) == ref.ggml_type_size(t), t
        assert rt.ggml_blck_size(t) == ref.ggml_blck_size(t), t
        assert rt.ggml_type_name(t) == ref.ggml_type_name(t), t
    for op in range(76):
        assert rt.ggml_op_name(op) == ref.ggml_op_name(op), op
    assert rt.ggml_tensor_overhead() == ref.ggml_tensor_overhead()
    assert rt.ggml_graph_overhead() == ref.ggml_graph_overhead()
    for n in (16, 100, 2048, 8192):
        assert rt.ggml_graph_overhead_custom(n, False) == ref.ggml_graph_overhead_custom(n, False)


@needs_ref
def test_fp16_conversion_matches_reference(rt, ref):
    G.Context(ref, 1024).free()  # the reference fills its fp16 table in the first ggml_init
    for h in list(range(0, 65536, 7)) + [0x7c00, 0xfc00, 0x7e00, 0x0001, 0x03ff, 0x0400, 0x8001]:
        a, b = rt.ggml_fp16_to_fp32(h), ref.ggml_fp16_to_fp32(h)
        assert (np.isnan(a) and np.isnan(b)) or a == b, h
    vals = np.concatenate([synth.uniform(7, 4000) * 70000, synth.uniform(8, 2000) * 1e-4, synth.uniform(9, 2000) * 1e-7,
                           np.array([65504, 65519.99, 65520, 65536, 6.1e-5, 5.96e-8, 2.98e-8, 0, -0.0], np.float32)])
    for v in vals.astype(np.float32):
        assert rt.ggml_fp32_to_fp16(float(v)) == ref.ggml_fp32_to_fp16(float(v)), v


SMALL = [c for c in golden_cases(large=False) if c["type"] != 0]


@pytest.mark.parametrize("c", SMALL, ids=[c["name"] for c in SMALL])
def test_runtime_quantize_chunk_bit_exact(rt, c):
    K, N = c["K"], c["N"]
    w = synth.uniform(c["wseed"], K * N)
    out = np.empty(G.row_size(c["type"], K) * N, np.uint8)
    n = rt.ggml_quantize_chunk(c["type"], w.ctypes.data, out.ctypes.data, 0, N, K, None)
    assert n == out.nbytes
    if os.environ.get("GGML_MI355X_CORE_LIB"):
        # an instrumented build (tools/sanitize.sh): the quantizers' bytes follow gcc's FMA
        # contraction of the release flags, which instrumentation can change; memory checks only
        return
    ref = golden_blob(c["name"] + ".wq.bin")
    assert np.array_equal(out, ref), f"{np.count_nonzero(out != ref)} bytes differ"


def _graph_signature(lib):
    """A GPT-2-block-like graph; returns (ops, shapes, strides, op_params) in node order."""
    with G.Context(lib, 256 * lib.ggml_tensor_overhead() + lib.ggml_graph_overhead(), no_alloc=True) as c:
        ctx = c.ctx
        n_embd, n_tok, n_head = 64, 5, 4
        x = lib.ggml_new_tensor_2d(ctx, 0, n_embd, n_tok)
        w = lib.ggml_new_tensor_2d(ctx, 12, 256, 3 * n_embd)
        wx = lib.ggml_new_tensor_2d(ctx, 1, n_embd, 3 * n_embd)
        g = lib.ggml_new_tensor_1d(ctx, 0, n_embd)
        cur = lib.ggml_norm(ctx, x, 1e-5)
        cur = lib.ggml_add(ctx, lib.ggml_mul(ctx, cur, g), g)
        cur = lib.ggml_mul_mat(ctx, wx, cur)
        q = lib.ggml_view_2d(ctx, cur, n_embd, n_tok, cur.contents.nb[1], 0)
        k = lib.ggml_view_2d(ctx, cur, n_embd, n_tok, cur.contents.nb[1], 4 * n_embd)
        Q = lib.ggml_permute(ctx, lib.ggml_reshape_3d(ctx, lib.ggml_cont(ctx, q), n_embd // n_head, n_head, n_tok), 0, 2, 1, 3)
        Kt = lib.ggml_permute(ctx, lib.ggml_reshape_3d(ctx, lib.ggml_cont(ctx, k), n_embd // n_head, n_head, n_tok), 0, 2, 1, 3)
        kq = lib.ggml_mul_mat(ctx, Kt, Q)
        kq = lib.ggml_soft_max(ctx, lib.ggml_diag_mask_inf(ctx, lib.ggml_scale(ctx, kq, 0.125), 0))
        out = lib.ggml_gelu(ctx, lib.ggml_cont(ctx, lib.ggml_transpose(ctx, kq)))
        x4 = lib.ggml_new_tensor_2d(ctx, 0, 256, 2)
        out2 = lib.ggml_mul_mat(ctx, w, x4)
        gr = lib.ggml_new_graph(ctx)
        lib.ggml_build_forward_expand(gr, out)
        lib.ggml_build_forward_expand(gr, out2)
        gg = gr.contents
        sig = []
        for i in range(gg.n_nodes):
            t = gg.nodes[i].contents
            sig.append((t.op, tuple(t.ne), tuple(t.nb), tuple(t.op_params), t.type, t.name))
        return gg.n_nodes, gg.n_leafs, sig


@needs_ref
def test_graph_construction_matches_reference(rt, ref):
    assert _graph_signature(rt) == _graph_signature(ref)


def test_host_buffer_roundtrip_and_gallocr(rt):
    buft = rt.ggml_backend_cpu_buffer_type()
    with G.Context(rt, 64 * rt.ggml_tensor_overhead() + rt.ggml_graph_overhead(), no_alloc=True) as c:
        a = rt.ggml_new_tensor_2d(c.ctx, 0, 37, 5)
        b = rt.ggml_new_tensor_1d(c.ctx, 12, 512)
        buf = rt.ggml_backend_alloc_ctx_tensors_from_buft(c.ctx, buft)
        assert buf and rt.ggml_backend_buffer_is_host(buf)
        x = synth.uniform(3, 37 * 5)
        G.tensor_set(rt, a, x)
        assert np.array_equal(G.tensor_get(rt, a), x)
        assert b.contents.data % 32 == 0
        rt.ggml_backend_buffer_free(buf)
    # graph allocator: live ranges must not overlap
    with G.Context(rt, 64 * rt.ggml_tensor_overhead() + rt.ggml_graph_overhead(), no_alloc=True) as c:
        x = rt.ggml_new_tensor_2d(c.ctx, 0, 128, 4)
        t = x
        chain = []
        for i in range(6):
            t = rt.ggml_scale(c.ctx, t, 2.0)
            chain.append(t)
        y = rt.ggml_add(c.ctx, chain[-1], chain[1])
        g = rt.ggml_new_graph(c.ctx)
        rt.ggml_build_forward_expand(g, y)
        ga = rt.ggml_gallocr_new(buft)
        assert rt.ggml_gallocr_alloc_graph(ga, g)
        size = rt.ggml_gallocr_get_buffer_size(ga, 0)
        assert 0 < size < 9 * 128 * 4 * 4
        nodes = [g.contents.nodes[i].contents for i in range(g.contents.n_nodes)]
        spans = [(n.data, n.data + 128 * 4 * 4) for n in nodes]
        # chain[1] is live until the final add: nothing allocated after it may overlap it
        c1 = spans[1]
        for s in spans[2:-1]:
            assert s[1] <= c1[0] or s[0] >= c1[1]
        assert x.contents.data is not None
        rt.ggml_gallocr_free(ga)
