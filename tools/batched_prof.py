"""main-batched.cpp's decode loop (8 sequences) for a kernel trace: 24 steps after warm-up."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ggml-imax_amd"))
import numpy as np
from ggml_mi355x import ggml as G, gpt2
lib = G.runtime(); be = G.mi355x_backend(lib)
npar = 8
m = gpt2.Model(lib, gpt2.ensure_model(), be, n_ctx=512, n_batch=8)
prompt = m.tokenize("Once upon a time the cat sat on the mat and the dog ran away")[:8]
lg = m.decode_batch(prompt, list(range(8)), [0] * 8, all_logits=False)
for s in range(1, npar):
    m.kv_seq_cp(0, s, -1, -1)
nxt = [int(np.argmax(lg[-1]))] * npar
for t in range(28):
    lg = m.decode_batch(nxt, [8 + t] * npar, list(range(npar)))
    nxt = [int(v) for v in np.argmax(lg, axis=1)]
print("launches per step", lib.ggml_backend_mi355x_last_launch_count(be))
