"""One Q4_K 4096^2 GEMV per graph (32 rotated weights, bench's q4_K_4096x4096_single_graph) under
mmv_blocks settings, alternating: python tools/lone_gemv_blocks.py 0 384 512 768"""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "ggml-imax_amd"))
import bench  # noqa: E402
from ggml_mi355x import ggml as G  # noqa: E402
import torch  # noqa: E402

lib = G.runtime()
be = G.mi355x_backend(lib, 0)
sp = lib.ggml_backend_mi355x_get_stream(be)
w1 = bench.RotatedSingle(lib, be, 12, 4096, 4096, 1, 32)
for rep in range(3):
    line = []
    for b in [int(v) for v in sys.argv[1:]] or [0]:
        lib.ggml_backend_mi355x_set_tuning(b"mmv_blocks", b)
        for _ in range(64):
            w1.step()
        lib.ggml_backend_synchronize(be)
        ms = bench.event_time_per_step(torch, w1, sp, iters=256)
        line.append(f"blocks={b}: {ms * 1e3:.2f} us")
    print("  ".join(line), flush=True)
lib.ggml_backend_mi355x_set_tuning(b"mmv_blocks", 0)
w1.free()
lib.ggml_backend_free(be)
