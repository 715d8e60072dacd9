"""A LLaMA-shaped transformer block end to end on MI355X against the reference CPU (SURVEY.md
section 8 f4: RMSNorm / RoPE for LLaMA-shaped graphs; VERDICT r03 missing item 5).

The block is the LLaMA graph of this ggml era (llama.cpp build_llama without a KV cache): rms_norm ->
mul(attn_norm) -> Q / K / V Q4_K mul_mats -> RoPE (mode 0) -> KQ -> scale -> diag_mask_inf ->
soft_max -> KQV -> merge -> output projection + residual -> rms_norm -> mul(ffn_norm) -> gate / up
Q4_K mul_mats -> SiLU(gate) * up -> down projection + residual. Both sides build the same graph
through the same ggml calls on the same Q4_K bytes (quantized by the runtime's ggml_quantize_chunk,
byte-identical to the reference's).

* T = 5 tokens (the decode path, B <= 8): the backend's default settings run a graph whose quantized
  mul_mats consume computed values in the reference CPU's order, so the block is bit-identical.
* T = 16, 96, 200 tokens (the prompt path): under the default settings the quantized prompt
  mul_mats run the reference-order GEMV too, so the block is bit-identical at any length. The
  opt-out (ord_prefill_cols 0) sends them to the exact int8-MFMA GEMM: every mul_mat within 1e-5 of
  the reference, but each Q4_K mul_mat re-quantizes its input (Q8_K), which turns an ulp into a
  quant step; that path is held to the reference harness's NMSE 5e-4 (test-backend-ops).
"""
import os

import numpy as np
import pytest

from conftest import REPO
from ggml_mi355x import ggml as G
from ggml_mi355x import synth

REF_LIB = os.path.join(REPO, "oracle", "_ref", "libggml_ref.so")
pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not os.path.exists(REF_LIB), reason="make -C oracle ref")]

F32, I32, Q4_K = G.GGML_TYPE_F32, G.GGML_TYPE_I32, 12
E, H, FF = 512, 4, 1536
D = E // H


def _weights():
    rt = G.runtime()
    w = {}
    for i, (name, k, n) in enumerate((("wq", E, E), ("wk", E, E), ("wv", E, E), ("wo", E, E), ("w1", E, FF), ("w3", E, FF),
                                      ("w2", FF, E))):
        f = (synth.uniform(100 + i, k * n) * np.float32(0.08)).astype(np.float32)
        out = np.empty(G.row_size(Q4_K, k) * n, np.uint8)
        rt.ggml_quantize_chunk(Q4_K, f.ctypes.data, out.ctypes.data, 0, n, k, None)
        w[name] = (out, k, n)
    w["attn_norm"] = (1.0 + 0.1 * synth.uniform(120, E)).astype(np.float32)
    w["ffn_norm"] = (1.0 + 0.1 * synth.uniform(121, E)).astype(np.float32)
    return w


def _build(L, c, W, T, x, pos):
    feeds = []

    def new(t, arr, *ne):
        fn = {1: L.ggml_new_tensor_1d, 2: L.ggml_new_tensor_2d}[len(ne)]
        tt = fn(c, t, *ne)
        feeds.append((tt, arr))
        return tt

    xt = new(F32, x, E, T)
    pt = new(I32, pos, T)
    wt = {k: new(Q4_K, v[0], v[1], v[2]) for k, v in W.items() if k.startswith("w")}
    an = new(F32, W["attn_norm"], E)
    fn_ = new(F32, W["ffn_norm"], E)
    h = L.ggml_mul(c, L.ggml_rms_norm(c, xt, 1e-5), an)
    q = L.ggml_mul_mat(c, wt["wq"], h)
    k = L.ggml_mul_mat(c, wt["wk"], h)
    v = L.ggml_mul_mat(c, wt["wv"], h)
    q = L.ggml_rope(c, L.ggml_reshape_3d(c, q, D, H, T), pt, D, 0, 0)
    k = L.ggml_rope(c, L.ggml_reshape_3d(c, k, D, H, T), pt, D, 0, 0)
    Q = L.ggml_permute(c, q, 0, 2, 1, 3)
    K = L.ggml_permute(c, k, 0, 2, 1, 3)
    kq = L.ggml_mul_mat(c, K, Q)
    kq = L.ggml_soft_max(c, L.ggml_diag_mask_inf(c, L.ggml_scale(c, kq, float(1.0 / np.sqrt(D))), 0))
    V = L.ggml_cont(c, L.ggml_permute(c, L.ggml_reshape_3d(c, v, D, H, T), 1, 2, 0, 3))
    kqv = L.ggml_mul_mat(c, V, kq)
    cur = L.ggml_cont_2d(c, L.ggml_permute(c, kqv, 0, 2, 1, 3), E, T)
    out = L.ggml_add(c, L.ggml_mul_mat(c, wt["wo"], cur), xt)
    h2 = L.ggml_mul(c, L.ggml_rms_norm(c, out, 1e-5), fn_)
    g = L.ggml_mul_mat(c, wt["w1"], h2)
    u = L.ggml_mul_mat(c, wt["w3"], h2)
    y = L.ggml_add(c, L.ggml_mul_mat(c, wt["w2"], L.ggml_mul(c, L.ggml_silu(c, g), u)), out)
    return feeds, y


@pytest.fixture(scope="module")
def libs():
    rt = G.runtime()
    be = G.mi355x_backend(rt)
    ref = G.Lib([REF_LIB], isolated=True)
    cpu = ref.ggml_backend_cpu_init()
    ref.ggml_backend_cpu_set_n_threads(cpu, min(16, os.cpu_count() or 1))
    yield rt, be, ref, cpu
    ref.ggml_backend_free(cpu)
    rt.ggml_backend_free(be)


def _run(libs, T, seed=7):
    rt, be, ref, cpu = libs
    W = _weights()
    x = (synth.uniform(seed, E * T) * np.float32(2.0)).astype(np.float32)
    pos = (np.arange(T, dtype=np.int32) + 3).astype(np.int32)
    a = G.graph_once(rt, be, lambda c: _build(rt, c, W, T, x, pos), n_tensors=96)
    launches = rt.ggml_backend_mi355x_last_launch_count(be)
    b = G.graph_once(ref, cpu, lambda c: _build(ref, c, W, T, x, pos), n_tensors=96)
    nmse = float(np.sum((a - b) ** 2) / np.sum(b ** 2))
    rel = float(np.max(np.abs(a - b)) / np.max(np.abs(b)))
    print(f"T={T}: {launches} kernel launches, NMSE {nmse:.2e}, max rel {rel:.2e}, identical {float(np.mean(a == b)):.4f}")
    return a, b, nmse, rel


def test_llama_block_decode_path_bit_identical(libs):
    a, b, _, _ = _run(libs, 5)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_llama_block_prompt_path_bit_identical(libs):
    """T = 16 under the default settings: the graph's quantized mul_mats consume computed values,
    so it runs in the reference order, and its 16-column Q4_K mul_mats take the reference-order GEMV
    in 8-column chunks (ord_prefill_cols): the block output is the reference CPU's bits."""
    a, b, _, _ = _run(libs, 16)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.mark.parametrize("T", [96, 200])
def test_llama_block_long_prompt_bit_identical(libs, T):
    """Prompts past 64 tokens under the default settings (round 6: the reference-order prompt path
    has no column limit): the Q/K/V and gate/up Q4_K mul_mats of 96 / 200 columns run the
    reference-order streaming GEMV, 8 columns per grouped member, so the whole block -- attention
    over T keys included -- is the reference CPU's bits."""
    a, b, _, _ = _run(libs, T)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_llama_block_prompt_path_mfma_within_tolerance(libs):
    """The opt-out (ord_prefill_cols 0): T = 16 through the exact int8-MFMA GEMMs -- the reference
    harness's NMSE 5e-4 on the block output and a max-rel bound. Each Q4_K mul_mat is within 1e-5 of
    the reference, but its input is re-quantized (Q8_K), which turns an f32 fold-order ulp into a
    quant step."""
    rt = libs[0]
    assert rt.ggml_backend_mi355x_set_tuning(b"ord_prefill_cols", 0)
    try:
        a, b, nmse, rel = _run(libs, 16)
    finally:
        rt.ggml_backend_mi355x_set_tuning(b"ord_prefill_cols", 2 ** 31 - 1)
    assert np.all(np.isfinite(a))
    assert nmse <= 5e-4
    assert rel <= 3e-2, rel
