"""GPT-2-117M f16 decode (bench.py's gpt2 leg) ms/token under backend tuning settings, each setting
run in turn: python tools/gpt2_tune.py f16_bn=5 f16_bn=15 ..."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "ggml-imax_amd"))
import bench  # noqa: E402
from ggml_mi355x import ggml as G  # noqa: E402

lib = G.runtime()
be = G.mi355x_backend(lib)
for spec in sys.argv[1:] or ["f16_bn=5"]:
    kv = [s.split("=") for s in spec.split(",")]
    old = {}
    for k, v in kv:
        assert lib.ggml_backend_mi355x_set_tuning(k.encode(), int(v)), k
    r = bench.gpt2_bench(lib, be, n_decode=96)
    print(f"{spec:40s} ms/token {r['ms_per_decode_token']:.4f}  launches {r.get('kernel_launches_per_token')}", flush=True)
lib.ggml_backend_free(be)
