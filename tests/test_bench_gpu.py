"""GPU checks of bench.py's multi-GPU helpers on a one-GPU box: torch views alias ggml device
memory (the zero-copy hand-off RCCL works on), and the tensor-split row leg (RCCL broadcast +
all-gather around the local GEMM) runs end to end as a single-rank RCCL job at the BASELINE
config 5 shape, whose reassembled output matches the reference CPU's golden columns element-wise
and equals the unsplit product bit for bit."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu

CHILD = r"""
import json, os, sys
sys.path.insert(0, os.environ["REPO"]); sys.path.insert(0, os.path.join(os.environ["REPO"], "ggml-imax_amd"))
import numpy as np, torch, torch.distributed as dist
import bench
from ggml_mi355x import ggml as G, synth
lib = G.runtime(); be = G.mi355x_backend(lib, 0); dev = torch.device("cuda", 0)
# 1) aliasing: a torch view of a ggml tensor sees tensor_set data and torch writes land in ggml
ctx = G.Context(lib, lib.ggml_tensor_overhead() * 4, no_alloc=True)
t = lib.ggml_new_tensor_1d(ctx.ctx, G.GGML_TYPE_F32, 1000)
buf = lib.ggml_backend_alloc_ctx_tensors(ctx.ctx, be)
v = synth.uniform(9, 1000); G.tensor_set(lib, t, v)
tv = bench.torch_view(torch, lib, t, dev)
alias_read = bool(np.array_equal(tv.cpu().numpy(), v))
tv.mul_(2.0); torch.cuda.synchronize()
alias_write = bool(np.array_equal(G.tensor_get(lib, t), v * 2))
lib.ggml_backend_buffer_free(buf); ctx.free()
# 2) the row-split leg as a 1-rank RCCL job
dist.init_process_group("nccl", init_method="tcp://127.0.0.1:" + os.environ["PORT"], rank=0, world_size=1, device_id=dev)
res, y_split = bench.rowsplit_prefill(lib, be, dist, 1, 0, dev, torch, steps=2, return_y=True)  # BASELINE config 5 shape
dist.destroy_process_group()
K, N, B = 4096, 4096, 512
wl = bench.MulMatWorkload(lib, be, 12, K, N, B, 1, seed=42)
G.tensor_set(lib, wl.x[0], synth.uniform(43, K * B))
wl.step(); lib.ggml_backend_synchronize(be)
direct = G.tensor_get(lib, wl.y[0]).reshape(B, N)
wl.free(); lib.ggml_backend_free(be)
same = bool(np.array_equal(direct.view(np.uint32), y_split.view(np.uint32)))
print(json.dumps({"alias_read": alias_read, "alias_write": alias_write, "res": res, "same_as_direct": same}))
"""


def test_torch_view_and_rowsplit_leg():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, REPO=REPO, PORT=str(port))
    p = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert out["alias_read"] and out["alias_write"]
    assert "error" not in out["res"], out["res"]
    assert out["res"]["rows_per_rank"] == 4096
    # element-wise: the reference CPU's own output for this workload (tests/golden, config 5) ...
    assert out["res"]["parity_ok"], out["res"]
    # ... and bit for bit the unsplit product
    assert out["same_as_direct"]


def test_bench_two_ranks_rehearsal():
    """bench.py's world > 1 branches end to end before the driver's 8-GPU run: two ranks launched by
    torch.distributed.run as the driver launches them, sharing this box's one GPU over the gloo
    collective backend (BENCH_DIST_BACKEND; RCCL refuses two ranks on one device). Checks the
    barrier + max-over-ranks timing, the whole-job value (both ranks' units), and the config-5
    prompt-sharded prefill leg (256 columns per rank); the RCCL row-split leg reports that it needs
    RCCL instead of failing the line."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, BENCH_DIST_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
           "--master-port", str(port), os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1", "--no-gpt2",
           "--no-cpu"]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=400, cwd=REPO)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-3000:])
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]  # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 3 and out["scaling"] == "weak"
    assert out["value"] > 0 and out["ms_per_step"] > 0
    pf = out["prefill_sharded"]
    assert pf["columns_per_rank"] == 256 and pf["us_per_mul_mat"] > 0
    assert "RCCL" in out["prefill_rowsplit_rccl"].get("error", "")
