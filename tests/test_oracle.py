"""Pin the CPU restatement (oracle/) against the reference's own golden vectors.

The fixtures were produced by the real reference build (oracle/_ref, see
tests/golden/make_golden.py). Quantize / dequantize / activation quantization must be
bit-exact; mul_mat outputs within float summation-order error.
"""
import hashlib
import os

import numpy as np
import pytest

from conftest import golden_blob, golden_cases
import pyoracle as orc
from ggml_mi355x import synth

SMALL = golden_cases(large=False)
LARGE = golden_cases(large=True)


def _inputs(c):
    K, N, B = c["K"], c["N"], c["B"]
    return synth.uniform(c["wseed"], K * N), synth.uniform(c["xseed"], K * B)


@pytest.mark.parametrize("c", SMALL, ids=[c["name"] for c in SMALL])
def test_weight_quantize_bit_exact(c):
    w, _ = _inputs(c)
    q = orc.quantize(c["type"], w, c["K"])
    ref = golden_blob(c["name"] + ".wq.bin")
    assert q.nbytes == ref.nbytes
    assert np.array_equal(q, ref), f"{np.count_nonzero(q != ref)} bytes differ"


@pytest.mark.parametrize("c", SMALL, ids=[c["name"] for c in SMALL])
def test_activation_quantize_bit_exact(c):
    if c["type"] == orc.F32:
        pytest.skip("f32 activations are used as-is")
    _, x = _inputs(c)
    vdt = orc.vec_dot_type(c["type"])
    q = orc.quantize_act(vdt, x, c["K"])
    ref = golden_blob(c["name"] + ".xq.bin")
    assert np.array_equal(q, ref), f"{np.count_nonzero(q != ref)} of {q.size} bytes differ"


@pytest.mark.parametrize("c", [c for c in SMALL if c["name"].startswith("s_") and c["type"] != 0],
                         ids=lambda c: c["name"])
def test_dequantize_bit_exact(c):
    K, N = c["K"], c["N"]
    wq = golden_blob(c["name"] + ".wq.bin")
    d = orc.dequantize(c["type"], wq, K * N)
    ref = golden_blob(c["name"] + ".wdq.f32", np.float32)
    assert np.array_equal(d.view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("c", SMALL, ids=[c["name"] for c in SMALL])
def test_mul_mat_matches_reference(c):
    K, N, B = c["K"], c["N"], c["B"]
    _, x = _inputs(c)
    wq = golden_blob(c["name"] + ".wq.bin")
    y = orc.mul_mat(c["type"], wq, K, N, x, B)
    ref = golden_blob(c["name"] + ".y.f32", np.float32)
    err = np.abs(y - ref).max() / max(np.abs(ref).max(), 1e-30)
    assert err <= 1e-5, err


@pytest.mark.parametrize("t", ["f16", "q4_0", "q8_0", "q4_K", "q5_K"])
def test_cos_data_quantize(t):
    """test-quantize-fns.cpp data (0.1 + 2 cos(i)): bit-exact bytes + its RMSE thresholds (:16-22)."""
    x = golden_blob("cos_input.f32", np.float32)
    ty = orc.TYPES_BY_NAME[t]
    q = orc.quantize(ty, x, x.size)
    assert np.array_equal(q, golden_blob(f"cos_{t}.wq.bin"))
    rt = orc.dequantize(ty, q, x.size)
    # the reference's "rmse" is sqrt(sum d^2) / n (test-quantize-fns.cpp:35-42), bound 0.002 (:17)
    d = (rt.astype(np.float64) - x.astype(np.float64))
    err = float(np.sqrt(np.sum(d * d)) / x.size)
    assert err < 0.002, err


@pytest.mark.slow
@pytest.mark.parametrize("c", LARGE, ids=[c["name"] for c in LARGE])
def test_large_weights_hash_and_output(c):
    K, N, B = c["K"], c["N"], c["B"]
    w, x = _inputs(c)
    q = orc.quantize(c["type"], w, K)
    assert hashlib.sha256(q.tobytes()).hexdigest() == c["wq_sha256"]
    if N * B <= 4096 * 8:
        y = orc.mul_mat(c["type"], q, K, N, x, B)
        ref = golden_blob(c["name"] + ".y.f32", np.float32)
        err = np.abs(y - ref).max() / np.abs(ref).max()
        assert err <= 1e-5, err


PREFILL = golden_cases(large=True, prefill=True)


@pytest.mark.parametrize("c", PREFILL, ids=[c["name"] for c in PREFILL])
def test_prefill_fixture_columns_vs_restatement(c):
    """The P_* fixtures (prefill-sized Y: SHA-256 + every step-th column) against the CPU
    restatement on those columns: same weight bytes, outputs within 1e-5."""
    K, N, B = c["K"], c["N"], c["B"]
    w, x = _inputs(c)
    q = orc.quantize(c["type"], w, K)
    assert hashlib.sha256(q.tobytes()).hexdigest() == c["wq_sha256"]
    step = c["y_col_step"]
    xs = np.ascontiguousarray(x.reshape(B, K)[::step])
    ys = golden_blob(c["name"] + ".ys.f32", np.float32).reshape(-1, N)
    y = orc.mul_mat(c["type"], q, K, N, xs.ravel(), xs.shape[0]).reshape(-1, N)
    err = np.abs(y - ys).max() / np.abs(ys).max()
    assert err <= 1e-5, err


def test_mul_mat_exact_plumbing():
    """tests/test-mul-mat.cpp:262-298 style: integer-valued f32 operands give exact results."""
    rng = np.random.default_rng(0)
    K, N, B = 36, 4, 16
    w = rng.integers(-4, 5, size=K * N).astype(np.float32)
    x = rng.integers(-4, 5, size=K * B).astype(np.float32)
    y = orc.mul_mat(orc.F32, w, K, N, x, B).reshape(B, N)
    exp = x.reshape(B, K) @ w.reshape(N, K).T
    assert np.array_equal(y, exp)
