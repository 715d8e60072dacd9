"""Quantized GPT-2-117M decode (bench.py's gpt2_q4_k leg, default settings: reference order) ms/token
under backend tuning settings, alternating over `passes` rounds:
python tools/gpt2q_tune.py q4_k 3 mmv_pro4=1 mmv_pro4=0"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "ggml-imax_amd"))
import bench  # noqa: E402
from ggml_mi355x import ggml as G  # noqa: E402
from ggml_mi355x import gpt2  # noqa: E402

lib = G.runtime()
be = G.mi355x_backend(lib)
qt, passes, specs = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
path = gpt2.ensure_quantized_model(lib, qt)
for p in range(passes):
    for spec in specs:
        kv = [s.split("=") for s in spec.split(",")]
        for k, v in kv:
            assert lib.ggml_backend_mi355x_set_tuning(k.encode(), int(v)), k
        r = bench.gpt2_bench(lib, be, n_decode=96, path=path)
        print(f"pass {p} {qt} {spec:30s} ms/token {r['ms_per_decode_token']:.4f}  launches {r.get('kernel_launches_per_token')}", flush=True)
lib.ggml_backend_free(be)
