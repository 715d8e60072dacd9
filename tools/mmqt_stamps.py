"""k_mmqt phase timing from in-kernel s_memtime stamps (diagnostic build: `make -C ggml-imax_amd
diaglib`, GGML_MI355X_BACKEND_LIB=ggml-imax_amd/lib/diag/libggml_mi355x.so; results invalid).
Q4_K 4096 x 4096 x B (default 512): per K step of waves 0 (low half) and 4 (high half) of workgroups
0 and 97: cycles of the MFMA steps (with the next stage's DMAs behind them), the combine, the wait
for the DMAs, and the barrier. argv[2]: ablation bits (1 no weight DMAs, 2 no combine, 4 no DMAs;
7: the per-half synchronized form, mmq_long 3, without ablations)."""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "ggml-imax_amd"))
import bench  # noqa: E402
from ggml_mi355x import ggml as G  # noqa: E402

lib = G.runtime()
be = G.mi355x_backend(lib, 0)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
abl = int(sys.argv[2]) if len(sys.argv) > 2 else 0
assert lib.ggml_backend_mi355x_set_tuning(b"mmq_long", 16 + abl)
wl = bench.MulMatWorkload(lib, be, 12, 4096, 4096, B, 1)
for _ in range(20):
    wl.step()
lib.ggml_backend_synchronize(be)
raw = G.tensor_get(lib, wl.y[0]).view(np.uint64)[:320].reshape(2, 2, 80).astype(np.int64)
SK = 8
for wg in range(2):
    for half in range(2):
        t = raw[wg, half]
        t0 = t[0]
        tot = np.zeros(4, np.int64)
        rows = []
        for u in range(SK):
            a, b_, c, d = t[2 + 4 * u: 6 + 4 * u]
            nxt = t[2 + 4 * (u + 1)] if u + 1 < SK else d
            ph = np.array([b_ - a, c - b_, d - c, nxt - d])
            tot += ph
            rows.append(ph)
        print(f"workgroup {'0' if wg == 0 else '97'} wave {4 * half}: prologue {t[1] - t0}, steps {t[2 + 4 * SK - 1] - t[2]} (s_memtime units)")
        for u, ph in enumerate(rows):
            print(f"  step {u}: mfma+dma {ph[0]:6d}  combine {ph[1]:6d}  dma wait {ph[2]:6d}  barrier {ph[3]:6d}")
        print(f"  total: mfma+dma {tot[0]} combine {tot[1]} dma wait {tot[2]} barrier {tot[3]}")
lib.ggml_backend_mi355x_set_tuning(b"mmq_long", 0)
wl.free()
lib.ggml_backend_free(be)
