"""Batched decode (main-batched.cpp, 8 sequences) ms/step under backend tuning settings:
python tools/batched_tune.py f16_rgs=0 f16_rgs=2 f16_rgs=4 "f16_rgs=4,f16_waves=1024" ..."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "ggml-imax_amd"))
import bench  # noqa: E402
from ggml_mi355x import ggml as G  # noqa: E402

lib = G.runtime()
be = G.mi355x_backend(lib)
for spec in sys.argv[1:] or ["f16_rgs=0"]:
    kv = [s.split("=") for s in spec.split(",")]
    for k, v in kv:
        assert lib.ggml_backend_mi355x_set_tuning(k.encode(), int(v)), k
    r = bench.gpt2_batched_bench(lib, be, n_steps=24)
    print(f"{spec:40s} ms/step {r['ms_per_step']:.4f}  predict {r.get('ms_per_step_predict', 0):.4f}  launches {r['kernel_launches_per_step']}  "
          f"no-capture {r.get('no_graph_capture', {}).get('ms_per_step')}", flush=True)
    for k, v in kv:
        lib.ggml_backend_mi355x_set_tuning(k.encode(), 0)
lib.ggml_backend_free(be)
