"""Alternating A/B of the Q4_0 tree-order decode GEMV on the canonical blocks (q40r 0) and on the
16-byte-aligned repacked copy (q40r 1): the bench sweep's workload (R rotated weights, one grouped
launch per step), HIP events on the backend stream.
usage: python tools/q40r_ab.py [passes]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "ggml-imax_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
from ggml_mi355x import ggml as G  # noqa: E402

lib = G.runtime()
be = G.mi355x_backend(lib)
sp = lib.ggml_backend_mi355x_get_stream(be)
passes = int(sys.argv[1]) if len(sys.argv) > 1 else 3
shapes = [(4096, 4096, 1), (4096, 11008, 1), (4096, 4096, 2), (11008, 4096, 1)]
for K, N, B in shapes:
    R = max(8, int(320 * 2**20 // (G.row_size(2, K) * N)) + 1)
    w = bench.MulMatWorkload(lib, be, 2, K, N, B, R)
    res = {0: [], 1: []}
    for p in range(passes):
        for v in (0, 1):
            lib.ggml_backend_mi355x_set_tuning(b"q40r", v)
            for _ in range(3):
                w.step()
            lib.ggml_backend_synchronize(be)
            ms = bench.event_time_per_step(torch, w, sp, iters=10)
            res[v].append(R * bench.unit_bytes(2, K, N, B) / (ms / 1e3) / 1e9)
    lib.ggml_backend_mi355x_set_tuning(b"q40r", 1)
    w.free()
    fmt = lambda a: " ".join(f"{x:7.1f}" for x in a)
    print(f"q4_0 K={K:5d} N={N:5d} B={B} R={R:3d}  canonical GB/s {fmt(res[0])}  repacked GB/s {fmt(res[1])}", flush=True)
lib.ggml_backend_free(be)
