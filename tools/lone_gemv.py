"""One mul_mat per graph_compute (the dependent-layer shape), R rotated weight copies: HIP-event
time per graph and host time per graph_compute_async call, per (type, K, N, B).
usage: python tools/lone_gemv.py [type:K:N:B ...]   (default q4_K:4096:4096:1)
Env GGML_MI355X_* tunings pass through (e.g. GGML_MI355X_MMV_VARIANT)."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "ggml-imax_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
from ggml_mi355x import ggml as G  # noqa: E402

lib = G.runtime()
be = G.mi355x_backend(lib)
sp = lib.ggml_backend_mi355x_get_stream(be)
cases = sys.argv[1:] or ["q4_K:4096:4096:1"]
for case in cases:
    tn, K, N, B = case.split(":")
    t, K, N, B = bench.TYPE_NAMES[tn], int(K), int(N), int(B)
    R = max(8, int(320 * 2**20 // (G.row_size(t, K) * N)) + 1)
    w = bench.RotatedSingle(lib, be, t, K, N, B, R)
    for _ in range(2 * R):
        w.step()
    lib.ggml_backend_synchronize(be)
    ms = bench.event_time_per_step(torch, w, sp, iters=8 * R)
    # host cost of one call: the loop's host time with the device far behind (no sync inside)
    t0 = time.perf_counter()
    for _ in range(4 * R):
        w.step()
    host_us = (time.perf_counter() - t0) / (4 * R) * 1e6
    lib.ggml_backend_synchronize(be)
    ub = bench.unit_bytes(t, K, N, B)
    print(f"{case:22s} R={R:3d} us/graph {ms * 1e3:7.2f}  GB/s {ub / (ms / 1e3) / 1e9:8.1f}  host us/call {host_us:6.2f}  "
          f"launches {lib.ggml_backend_mi355x_last_launch_count(be)}", flush=True)
    w.free()
lib.ggml_backend_free(be)
