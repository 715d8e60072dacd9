"""Batched-prefill mul_mat timing (BASELINE config 5 shape) on MI355X: HIP-event time per
mul_mat for B in sys.argv (default 512 64), all weight types of the path."""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "ggml-imax_amd"))
import bench  # noqa: E402
from ggml_mi355x import ggml as G  # noqa: E402
import torch  # noqa: E402

lib = G.runtime()
be = G.mi355x_backend(lib, 0)
sp = lib.ggml_backend_mi355x_get_stream(be)
Bs = [int(b) for b in sys.argv[1:]] or [512, 64]
refs = {}
VARS = [int(v) for v in os.environ.get("MMQ_VARIANTS", "0").split(",")]
# PF_LONG: mmq_long settings to compare (Q4_K / Q5_K past 128 columns: 1 k_mmqw, 2 k_mmqt, 3-4 k_mmqs, 6 k_mmqt DMAs at step start)
LONGS = [int(v) for v in os.environ.get("PF_LONG", "0").split(",")]
VARS = [(v, l) for v in VARS for l in LONGS]
# PF_MMV_BLOCKS: decode GEMV grid targets to compare (0 = automatic)
BLOCKS = [int(v) for v in os.environ.get("PF_MMV_BLOCKS", "0").split(",")]
VARS = [(v, l, b) for (v, l) in VARS for b in BLOCKS]
# PF_PLANES: repacked-planes settings to compare (Q4_K / Q5_K past 128 columns: 1 k_mmqr, 0 the canonical kernels)
PLANES = [int(v) for v in os.environ.get("PF_PLANES", "0").split(",")]
VARS = [(v, l, b, p) for (v, l, b) in VARS for p in PLANES]
for tname in os.environ.get("PF_TYPES", "q4_K,q5_K,q4_0,q8_0,f16").split(","):
    for B in Bs:
      for var, lng, blk, pl in VARS:
        lib.ggml_backend_mi355x_set_tuning(b"planes", pl)
        lib.ggml_backend_mi355x_set_tuning(b"mmq_variant", var)
        lib.ggml_backend_mi355x_set_tuning(b"mmq_long", lng)
        lib.ggml_backend_mi355x_set_tuning(b"mmv_blocks", blk)
        t = bench.TYPE_NAMES[tname]
        R = int(os.environ.get("PF_R", "8"))  # weight copies per step (36 x 9.4 MB > the 256 MB Infinity Cache)
        wl = bench.MulMatWorkload(lib, be, t, 4096, 4096, B, R)
        for _ in range(3):
            wl.step()
        ms = np.median([bench.event_time_per_step(torch, wl, sp, iters=5) for _ in range(3)])
        torch.cuda.synchronize()
        # the same mul_mat, one per graph (R graphs round-robin: no grouping across mul_mats)
        ms1 = float("nan")
        if os.environ.get("PF_SINGLE", "1") != "0":
            one = bench.RotatedSingle(lib, be, t, 4096, 4096, B, R)
            for _ in range(R):
                one.step()
            ms1 = np.median([bench.event_time_per_step(torch, one, sp, iters=4 * R) for _ in range(3)])
            one.free()
        y = G.tensor_get(lib, wl.y[0])
        ref = refs.setdefault((tname, B), y)
        same = "bit-equal to the first variant" if np.array_equal(y.view(np.uint32), ref.view(np.uint32)) else "DIFFERS from the first variant"
        print(f"{tname:5s} B={B:4d} var={var:5d} long={lng} blocks={blk} planes={pl} R={R}: {ms * 1e3 / R:8.2f} us/mul_mat in a graph of {R}  {2 * 4096 * 4096 * B * R / (ms / 1e3) / 1e12:7.1f} TFLOP/s  "
              f"| one per graph {ms1 * 1e3:8.2f} us  {same}")
        wl.free()
lib.ggml_backend_free(be)
