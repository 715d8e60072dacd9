"""The reference CPU's summation order for Q4_0 / Q8_0 rows (what `k_mmv_q0_ord` replays on the GPU
in mmv_order=1, mmv.hip), restated in numpy and pinned against the reference CPU backend built
from /root/reference's sources (oracle/_ref): per block i, the AVX2 dot keeps eight float lanes l
(mul_sum_i8_pairs_float: the exact int32 sum of elements 4l..4l+3; Q4_0 after
bytes_from_nibbles_32 - 8) in acc[l] = fma(x.d * y.d, q, acc[l]) over the blocks in order, then
hsum_float_8 = ((a0 + a4) + (a2 + a6)) + ((a1 + a5) + (a3 + a7))
(ggml_vec_dot_q8_0_q8_0 src/ggml-quants.c:4819+, ggml_vec_dot_q4_0_q8_0 :3469+, hsum_float_8).
Test infrastructure only (CPU); rows of any block count, including K % 256 != 0."""
import os

import numpy as np
import pytest

from conftest import REPO
import pyoracle as orc
from ggml_mi355x import ggml as G
from ggml_mi355x import synth

REF_LIB = os.path.join(REPO, "oracle", "_ref", "libggml_ref.so")


def fma32(a, b, c):
    # a * b is exact in double (24 x 24 bits); one rounding of the double sum to f32 equals the
    # fused rounding unless the double sum itself rounded at a float tie (checked: not at these sizes)
    return np.float32(float(a) * float(b) + float(c))


def chain_mul_mat(tname, wq, xq, K, N, B):
    nb = K // 32
    bs = 34 if tname == "q8_0" else 18
    W = np.frombuffer(wq.tobytes(), np.uint8).reshape(N, nb * bs)
    X = np.frombuffer(xq.tobytes(), np.uint8).reshape(B, nb * 34)
    f32 = np.float32
    out = np.zeros((B, N), np.float32)
    for b in range(B):
        for n in range(N):
            A = [f32(0)] * 8
            for i in range(nb):
                wb = W[n, i * bs:(i + 1) * bs]
                xb = X[b, i * 34:(i + 1) * 34]
                d = f32(wb[:2].view(np.float16).astype(np.float32)[0] * xb[:2].view(np.float16).astype(np.float32)[0])
                xv = xb[2:].view(np.int8).astype(np.int64)
                if tname == "q8_0":
                    wv = wb[2:].view(np.int8).astype(np.int64)
                else:
                    qs = wb[2:].astype(np.int64)
                    wv = np.concatenate([qs & 15, qs >> 4]) - 8
                for l in range(8):
                    A[l] = fma32(d, int((wv[4 * l:4 * l + 4] * xv[4 * l:4 * l + 4]).sum()), A[l])
            r = [f32(A[l] + A[l + 4]) for l in range(4)]
            out[b, n] = f32(f32(r[0] + r[2]) + f32(r[1] + r[3]))
    return out


@pytest.mark.skipif(not os.path.exists(REF_LIB), reason="reference lib not built (make -C oracle ref)")
@pytest.mark.parametrize("tname", ["q4_0", "q8_0"])
@pytest.mark.parametrize("K,N,B", [(416, 24, 1), (384, 16, 3), (96, 9, 2)])
def test_q0_chain_restatement_matches_reference_cpu(tname, K, N, B):
    t = orc.TYPES_BY_NAME[tname]
    wq = orc.quantize(t, synth.uniform(11 + K + N, K * N), K)
    x = synth.uniform(12 + K + B, K * B)
    ref = G.Lib([REF_LIB], isolated=True)
    cpu = ref.ggml_backend_cpu_init()
    try:
        yr = G.mul_mat_once(ref, cpu, t, wq, K, N, x, B).reshape(B, N)
    finally:
        ref.ggml_backend_free(cpu)
    yc = chain_mul_mat(tname, wq, orc.quantize_act(orc.vec_dot_type(t), x, K), K, N, B)
    assert np.array_equal(yc.view(np.uint32), yr.view(np.uint32))
