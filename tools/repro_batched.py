import os, sys
sys.path.insert(0, "/root/repo/ggml-imax_amd"); sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo") + "/ggml-imax_amd")
import numpy as np
from ggml_mi355x import ggml as G, gpt2
lib = G.runtime(); be = G.mi355x_backend(lib)
m = gpt2.Model(lib, gpt2.ensure_model(), be, n_ctx=256, n_batch=8)
prompt = m.tokenize("Once upon a time the cat sat on the mat")[:8]
print("prompt", len(prompt), flush=True)
lg = m.decode_batch(prompt, list(range(len(prompt))), [0] * len(prompt), all_logits=False)
print("prompt done", lg.shape, flush=True)
m.kv_seq_cp(0, 1, -1, -1)
for t in range(4):
    lg = m.decode_batch([int(np.argmax(lg[-1]))] * 2, [len(prompt) + t] * 2, [0, 1])
    print("step", t, lg.shape, flush=True)
