"""k_mmqx phase timing from in-kernel s_memtime stamps (GGML_MI355X_MMQ_VARIANT=1024 build path;
results invalid). Q4_K 4096 x 4096 x B=512: per stage, cycles of the MFMA steps, the combine and
the barrier, for wave 0 of two workgroups."""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "ggml-imax_amd"))
import bench  # noqa: E402
from ggml_mi355x import ggml as G  # noqa: E402

lib = G.runtime()
be = G.mi355x_backend(lib, 0)
lib.ggml_backend_mi355x_set_tuning(b"mmq_variant", 1024 | int(os.environ.get("STAMP_VARIANT", "0")))
B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
wl = bench.MulMatWorkload(lib, be, 12, 4096, 4096, B, 1)
for _ in range(20):
    wl.step()
lib.ggml_backend_synchronize(be)
raw = G.tensor_get(lib, wl.y[0]).view(np.uint64)[:160].reshape(2, 80)
for w in range(2):
    t = raw[w].astype(np.int64)
    t0 = t[0]
    print(f"workgroup {'0' if w == 0 else '97'}: prologue {t[1] - t0} cycles")
    tot = [0, 0, 0, 0]
    for sb in range(16):
        a, b_, c, d = t[2 + 4 * sb: 6 + 4 * sb]
        prev = t[1] if sb == 0 else t[5 + 4 * (sb - 1)]
        ph = [a - prev, b_ - a, c - b_, d - c]
        tot = [x + y for x, y in zip(tot, ph)]
        print(f"  sb {sb:2d}: gap {ph[0]:6d}  mfma-steps {ph[1]:6d}  combine {ph[2]:6d}  barrier {ph[3]:6d}")
    print(f"  total: steps {tot[1]} combine {tot[2]} barrier {tot[3]} (s_memtime units), end-start {t[5 + 60] - t0}")
rt = G.tensor_get(lib, wl.y[0]).view(np.uint64)[160:160 + 2 * 256].reshape(256, 2).astype(np.int64)
t0 = rt[:, 0].min()
st, en = (rt[:, 0] - t0) / 100.0, (rt[:, 1] - t0) / 100.0  # us (100 MHz)
print(f"workgroups: start spread {st.min():.2f}..{st.max():.2f} us, duration median {np.median(en - st):.2f} us "
      f"(min {np.min(en - st):.2f}, max {np.max(en - st):.2f}), last end {en.max():.2f} us")
order = np.argsort(st)
print("start times (us) of workgroups in start order, every 16th:", [round(float(st[i]), 2) for i in order[::16]])
lib.ggml_backend_mi355x_set_tuning(b"mmq_variant", 0)
wl.free()
lib.ggml_backend_free(be)
