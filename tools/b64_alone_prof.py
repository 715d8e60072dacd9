"""Config-5 per-GPU shard alone in its graph (Q4_K 4096^2 x B=64, one mul_mat per graph over 32
rotated weights): run under rocprofv3 --kernel-trace to split each graph into the activation
quantizer, the GEMM and the gaps (tools/b64_split.py reads the trace)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "ggml-imax_amd"))
import bench  # noqa: E402
from ggml_mi355x import ggml as G  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
lib = G.runtime()
be = G.mi355x_backend(lib)
w = bench.RotatedSingle(lib, be, 12, 4096, 4096, B, 32)
for _ in range(64):
    w.step()
lib.ggml_backend_synchronize(be)
for _ in range(128):
    w.step()
lib.ggml_backend_synchronize(be)
print("launches per graph", lib.ggml_backend_mi355x_last_launch_count(be))
w.free()
lib.ggml_backend_free(be)
