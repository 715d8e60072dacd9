"""Per-superblock timeline of the planes prefill kernel k_mmqr (diagnostic build: make -C
ggml-imax_amd diaglib): one Q4_K 4096^2 x B mul_mat group (R rotated weights), mmq_long 24.
Per workgroup wave 0 stamps s_memrealtime (10 ns ticks) at entry, after the prologue and per
superblock at step start / MFMAs issued / combine done / past the end-of-step wait. Prints medians
over workgroups of each phase and the workgroup span."""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("GGML_MI355X_BACKEND_LIB", os.path.join(REPO, "ggml-imax_amd", "lib", "diag", "libggml_mi355x.so"))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "ggml-imax_amd"))
import bench  # noqa: E402
from ggml_mi355x import ggml as G  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
R = int(sys.argv[2]) if len(sys.argv) > 2 else 16
SLOTS = 16 << 20
lib = G.runtime()
assert lib.ggml_backend_mi355x_stamps_enable(SLOTS), "diagnostic build needed"
be = G.mi355x_backend(lib)
wl = bench.MulMatWorkload(lib, be, 12, 4096, 4096, B, R)
for _ in range(3):
    wl.step()
lib.ggml_backend_synchronize(be)
assert lib.ggml_backend_mi355x_set_tuning(b"mmq_long", 24)
lib.ggml_backend_mi355x_stamps_reset()
wl.step()
lib.ggml_backend_synchronize(be)
words = np.zeros(SLOTS, np.uint64)
log = ctypes.create_string_buffer(1 << 20)
lib.ggml_backend_mi355x_stamps_read(words.ctypes.data, SLOTS, log, len(log))
S = 16
ns = ((4 * S + 2 + 7) // 8) * 8
for line in log.value.decode().splitlines():
    name, nb, off = line.split()
    if name != "k_mmqr":
        continue
    nb, off = int(nb), int(off)
    wgs = nb * 8 // ns
    st = words[off:off + wgs * ns].reshape(wgs, ns).astype(np.int64)
    t0 = st[:, 0].min()
    print(f"{wgs} workgroups; kernel span {(st[:, 5 + 4 * (S - 1)].max() - t0) / 100:.2f} us; "
          f"entry spread {(st[:, 0].max() - t0) / 100:.2f} us")
    print(f"prologue (entry -> first step) median {np.median(st[:, 1] - st[:, 0]) / 100:.3f} us")
    for sb in range(S):
        b = 2 + 4 * sb
        mf = np.median(st[:, b + 1] - st[:, b]) / 100
        cb = np.median(st[:, b + 2] - st[:, b + 1]) / 100
        wt = np.median(st[:, b + 3] - st[:, b + 2]) / 100
        print(f"sb {sb:2d}: mfma {mf:6.3f}  combine {cb:6.3f}  wait+barrier {wt:6.3f} us")
    first = st[:256]
    print(f"first 256 WGs: entry->exit median {np.median(first[:, 5 + 4 * (S - 1)] - first[:, 0]) / 100:.2f} us")
    break
wl.free()
lib.ggml_backend_free(be)
