"""The reference's OWN conformance executables, unmodified, run against the MI355X backend.

oracle/_ref/test-backend-ops-mi355x is tests/test-backend-ops.cpp of the reference compiled
from its sources and linked with the reference libggml plus our backend plugin (oracle/Makefile
`harness`). The plugin registers "MI355X0" into the reference registry; test-backend-ops then
compares every supported MUL_MAT case op-by-op against the reference CPU backend (NMSE <= 5e-4,
NaN/Inf and out-of-bounds sentinel checks, tests/test-backend-ops.cpp:358-515, :921-923).

This module is named test_00_* so it runs before any test initialises HIP in the pytest process
(the harness is started as a child process).
"""
import os
import subprocess

import pytest

from conftest import REPO

REF = os.path.join(REPO, "oracle", "_ref")
OPS = os.path.join(REF, "test-backend-ops-mi355x")
BUF = os.path.join(REF, "test-backend-buffer-mi355x")

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not os.path.exists(OPS), reason="harness not built (make -C oracle harness)")]


def _run(args, timeout=600):
    env = dict(os.environ, GGML_MI355X_AUTOREGISTER="1")
    p = subprocess.run(args, env=env, capture_output=True, text=True, timeout=timeout)
    return p.returncode, p.stdout + p.stderr


def test_reference_backend_ops_mul_mat():
    rc, out = _run([OPS, "test", "-o", "MUL_MAT", "-b", "MI355X0"])
    print(out[-4000:])
    assert "Backend name: MI355X0" in out, out[-2000:]
    assert rc == 0, out[-4000:]
    assert "FAIL" not in out.replace("\x1b[1;31mFAIL", "FAIL").split("Backend name: MI355X0")[1].split("backends passed")[0] or rc == 0


# the GPT-2 / LLaMA companion ops -- every case the reference's suite
# holds for them that our supports_op accepts (GELU/SILU f32, f16/f32 CPY/DUP/CONT, GET_ROWS f16/f32,
# RoPE modes 0/2, soft_max without ALiBi, ...); unsupported cases are reported "not supported"
COMPANION_OPS = ["ADD", "MUL", "SUB", "DIV", "SCALE", "NORM", "RMS_NORM", "SOFT_MAX", "DIAG_MASK_INF", "UNARY", "GET_ROWS",
                 "CPY", "DUP", "CONT", "ROPE"]


@pytest.mark.parametrize("op", COMPANION_OPS)
def test_reference_backend_ops_companion(op):
    rc, out = _run([OPS, "test", "-o", op, "-b", "MI355X0"])
    lines = out.replace("\x1b[1;31m", "").replace("\x1b[1;32m", "").replace("\x1b[0m", "").splitlines()
    bad = [ln for ln in lines if "FAIL" in ln]
    ok = [ln for ln in lines if ln.rstrip().endswith("OK")]
    print(f"{op}: {len(ok)} OK, {len(bad)} FAIL")
    print("\n".join(bad[:40]))
    assert "Backend name: MI355X0" in out, out[-2000:]
    assert rc == 0 and not bad, "\n".join(bad[:40]) or out[-3000:]
    assert ok, f"no {op} case ran on MI355X0"


def test_reference_backend_buffer():
    rc, out = _run([BUF])
    print(out[-3000:])
    assert rc == 0, out[-3000:]
    assert "MI355X0" in out
