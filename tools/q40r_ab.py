"""Alternating A/B of the Q4_0 / Q8_0 tree-order decode GEMV on the canonical blocks (knob 0) and on the
16-byte-aligned repacked copy (knob 1): the bench sweep's workload (R rotated weights, one grouped
launch per step), HIP events on the backend stream.
usage: python tools/q40r_ab.py [passes] [type] (type q4_0 -> knob q40r, q8_0 -> q80r)"""
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
tname = sys.argv[2] if len(sys.argv) > 2 else "q4_0"
T = bench.TYPE_NAMES[tname]
knob = b"q40r" if tname == "q4_0" else b"q80r"
shapes = [(4096, 4096, 1), (4096, 11008, 1), (11008, 4096, 1)]
for K, N, B in shapes:
    R = max(8, int(320 * 2**20 // (G.row_size(T, K) * N)) + 1)
    w = bench.MulMatWorkload(lib, be, T, K, N, B, R)
    res = {0: [], 1: []}
    for p in range(passes):
        for v in (0, 1):
            lib.ggml_backend_mi355x_set_tuning(knob, v)
            for _ in range(3):
                w.step()
            lib.ggml_backend_synchronize(be)
            ms = bench.event_time_per_step(torch, w, sp, iters=10)
            res[v].append(R * bench.unit_bytes(T, K, N, B) / (ms / 1e3) / 1e9)
    lib.ggml_backend_mi355x_set_tuning(knob, 1)
    w.free()
    fmt = lambda a: " ".join(f"{x:7.1f}" for x in a)
    print(f"{tname} K={K:5d} N={N:5d} B={B} R={R:3d}  canonical GB/s {fmt(res[0])}  repacked GB/s {fmt(res[1])}", flush=True)
lib.ggml_backend_free(be)
