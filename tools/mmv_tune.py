#!/usr/bin/env python3
"""Interleaved A/B of the fused GEMV launch variants in ONE process (cdna guide §5.4 rule 24).

usage: python tools/mmv_tune.py --variants 10:1024,21:1024 [--rounds 7] [--type q4_K --K 4096 --N 4096]
Prints median / min HIP-event time per step (R rotated mul_mats) and GB/s for each variant.
"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "ggml-imax_amd"))

import bench  # noqa: E402
from ggml_mi355x import ggml as G  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", required=True)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--type", default="q4_K")
    ap.add_argument("--K", type=int, default=4096)
    ap.add_argument("--N", type=int, default=4096)
    ap.add_argument("--B", type=int, default=1)
    ap.add_argument("--rotate", type=int, default=32)
    args = ap.parse_args()
    import torch

    lib = G.runtime()
    be = G.mi355x_backend(lib, 0)
    sp = lib.ggml_backend_mi355x_get_stream(be)
    t = bench.TYPE_NAMES[args.type]
    wl = bench.MulMatWorkload(lib, be, t, args.K, args.N, args.B, args.rotate)
    ub = bench.unit_bytes(t, args.K, args.N, args.B) * args.rotate
    variants = [tuple(int(x) for x in v.split(":")) for v in args.variants.split(",")]
    res = {v: [] for v in variants}
    for _ in range(3):
        wl.step()
    for r in range(args.rounds):
        for v in variants:
            lib.ggml_backend_mi355x_set_tuning(b"mmv_variant", v[0])
            lib.ggml_backend_mi355x_set_tuning(b"mmv_blocks", v[1])
            wl.step()
            res[v].append(bench.event_time_per_step(torch, wl, sp, iters=10))
    for v in variants:
        a = np.array(res[v])
        print(f"variant={v[0]:3d} blocks={v[1]:5d}: median {np.median(a) * 1e3:8.2f} us  min {a.min() * 1e3:8.2f} us  "
              f"-> {ub / (np.median(a) / 1e3) / 1e9:7.1f} GB/s (best {ub / (a.min() / 1e3) / 1e9:7.1f})")
    wl.free()
    lib.ggml_backend_free(be)


if __name__ == "__main__":
    main()
