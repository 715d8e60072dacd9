"""GPT-2 decode timing breakdown on MI355X (host build/alloc/compute split + tokens/s)."""
import ctypes, os, sys, time
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ggml-imax_amd"))
from ggml_mi355x import ggml as G, gpt2

n_decode = int(sys.argv[1]) if len(sys.argv) > 1 else 64
lib = G.runtime()
path = gpt2.ensure_quantized_model(lib, os.environ["GPT2_QTYPE"]) if os.environ.get("GPT2_QTYPE") else gpt2.ensure_model()
be = G.mi355x_backend(lib)
m = gpt2.Model(lib, path, be, n_ctx=1024, n_batch=8, host_io=os.environ.get("GPT2_HOST_IO", "1") == "1")
toks = m.tokenize("Once upon a time the cat sat on the mat and the dog ran away")[:32]
n_past = 0
for i in range(0, len(toks), 8):
    lg = m.eval(n_past, toks[i:i + 8]); n_past += len(toks[i:i + 8])
nxt = int(np.argmax(lg[-1]))
st = {"us_build": 0, "us_alloc": 0, "us_inputs": 0, "us_compute": 0, "us_launch": 0, "us_prebuild": 0, "us_wait": 0, "us_readback": 0}
t0 = time.perf_counter()
for _ in range(n_decode):
    lg = m.eval(n_past, [nxt], copy=False); n_past += 1
    nxt = int(np.argmax(lg[-1]))
    s = m.stats()
    for k in st: st[k] += s.get(k, 0)
dt = time.perf_counter() - t0
print(f"nodes/graph {s['nodes']}  decode {n_decode} tokens: {dt / n_decode * 1e3:.3f} ms/token = {n_decode / dt:.1f} tok/s")
print("per token us: " + ", ".join(f"{k}={v / n_decode:.1f}" for k, v in st.items()))
print("launches last graph:", lib.ggml_backend_mi355x_last_launch_count(be))
if hasattr(lib, "ggml_backend_mi355x_graph_stats"):
    gs = (ctypes.c_int64 * 4)()
    lib.ggml_backend_mi355x_graph_stats(be, gs)
    print("graph stats (captures, instantiations, updates, direct):", list(gs))
m.free()
lib.ggml_backend_free(be)
