"""Grouped decode GEMV (the bench sweep's shapes) GB/s under mmv_blocks settings, interleaved
twice: python tools/sweep_blocks.py 0 768 1536 2048"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "ggml-imax_amd"))
import bench  # noqa: E402
from ggml_mi355x import ggml as G  # noqa: E402
import torch  # noqa: E402

lib = G.runtime()
be = G.mi355x_backend(lib)
sp = lib.ggml_backend_mi355x_get_stream(be)
blocks = [int(b) for b in sys.argv[1:]] or [0]
shapes = [("q4_K", 12, 4096, 11008), ("q5_K", 13, 4096, 11008), ("q4_0", 2, 4096, 4096), ("q4_K", 12, 4096, 4096)]
wls = {}
for name, t, k, n in shapes:
    r = max(8, int(320 * 2**20 // (G.row_size(t, k) * n)) + 1)
    wls[(name, k, n)] = (bench.MulMatWorkload(lib, be, t, k, n, 1, r), r, t)
for rep in range(2):
    for b in blocks:
        lib.ggml_backend_mi355x_set_tuning(b"mmv_blocks", b)
        line = []
        for (name, k, n), (w, r, t) in wls.items():
            for _ in range(3):
                w.step()
            lib.ggml_backend_synchronize(be)
            ms = bench.event_time_per_step(torch, w, sp, iters=10)
            line.append(f"{name} {k}x{n}: {r * bench.unit_bytes(t, k, n, 1) / (ms / 1e3) / 1e9:7.1f} GB/s")
        print(f"blocks={b:5d}  " + "  ".join(line), flush=True)
lib.ggml_backend_mi355x_set_tuning(b"mmv_blocks", 0)
for w, _, _ in wls.values():
    w.free()
lib.ggml_backend_free(be)
