"""Batched decode (8 sequences): where a step's wall time goes -- the decode_batch call (launch, prebuild,
wait, logits copy) and the host argmax -- averaged over 48 steps."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ggml-imax_amd"))
import numpy as np
from ggml_mi355x import ggml as G, gpt2
lib = G.runtime(); be = G.mi355x_backend(lib)
npar = 8
m = gpt2.Model(lib, gpt2.ensure_model(), be, n_ctx=512, n_batch=8)
prompt = m.tokenize("Once upon a time the cat sat on the mat and the dog ran away")[:8]
for rep in range(2):
    m.kv_clear()
    lg = m.decode_batch(prompt, list(range(8)), [0] * 8, all_logits=False)
    for s in range(1, npar):
        m.kv_seq_cp(0, s, -1, -1)
    nxt = [int(np.argmax(lg[-1]))] * npar
    td = ta = 0.0
    for t in range(52):
        t0 = time.perf_counter()
        lg = m.decode_batch(nxt, [8 + t] * npar, list(range(npar)), copy=(rep == 0))
        t1 = time.perf_counter()
        nxt = [int(v) for v in np.argmax(lg, axis=1)]
        t2 = time.perf_counter()
        if t >= 4:
            td += t1 - t0
            ta += t2 - t1
    st = m.stats()
    print(f"copy={rep == 0} per step: decode_batch {td / 48 * 1e6:.1f} us, argmax {ta / 48 * 1e6:.1f} us; last call {st}", flush=True)
