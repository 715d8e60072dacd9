"""Decode GEMV throughput (grouped launches of R rotated weights, > 288 MiB per step) for the
BASELINE GEMV configs, one line per config: GB/s of algorithmic bytes by HIP events. Used for A/B
runs of two builds (GGML_MI355X_BACKEND_LIB) alternating on one box."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "ggml-imax_amd"))
import bench  # noqa: E402
from ggml_mi355x import ggml as G  # noqa: E402
import torch  # noqa: E402

lib = G.runtime()
be = G.mi355x_backend(lib, 0)
sp = lib.ggml_backend_mi355x_get_stream(be)
tag = sys.argv[1] if len(sys.argv) > 1 else ""
out = []
for name, tt, k, n in (("q4_K_4096x4096", 12, 4096, 4096), ("q4_0_4096x4096", 2, 4096, 4096), ("q4_K_4096x11008", 12, 4096, 11008),
                       ("q5_K_4096x11008", 13, 4096, 11008), ("q8_0_4096x11008", 8, 4096, 11008)):
    r = max(8, int(320 * 2**20 // (G.row_size(tt, k) * n)) + 1)
    if name == "q4_K_4096x4096":
        r = 32
    w = bench.MulMatWorkload(lib, be, tt, k, n, 1, r)
    for _ in range(3):
        w.step()
    lib.ggml_backend_synchronize(be)
    ms = min(bench.event_time_per_step(torch, w, sp, iters=10) for _ in range(3))
    out.append(f"{name} {r * bench.unit_bytes(tt, k, n, 1) / (ms / 1e3) / 1e9:7.1f}")
    w.free()
print(tag, " | ".join(out), flush=True)
lib.ggml_backend_free(be)
