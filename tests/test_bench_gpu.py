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
