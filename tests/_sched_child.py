"""Child process for tests/test_gpt2.py: the reference libggml (with its ggml_backend_sched), the
MI355X backend plugin and the GPT-2 driver built against the reference, all in one namespace
(RTLD_GLOBAL, no libggml_core in this process). Runs teacher-forced GPT-2 steps under the
reference scheduler with n_gpu_layers of the 12 layers on MI355X0 and the rest on the reference
CPU backend, and writes the logits of each configuration to <out>/<tag>.npy.

usage: python tests/_sched_child.py <model> <out_dir> <spec>[,<spec>...]
  spec = n_gpu_layers[:flags[:h]] -- flags = GPT2_SCHED_* bits (1 parallel scheduler with events,
  2 split inside a layer); h = persistent inputs in ggml_backend_mi355x_host_buffer_type() (pinned).
  Output file: <out_dir>/ngl<spec with ':' -> '_'>.npy
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ggml-imax_amd"))
from ggml_mi355x import ggml as G  # noqa: E402
from ggml_mi355x import gpt2  # noqa: E402

REF = os.path.join(REPO, "oracle", "_ref")


def main():
    model_path, out_dir, specs = sys.argv[1], sys.argv[2], sys.argv[3].split(",")
    layers = [int(v.split(":")[0]) for v in specs]
    lib = G.Lib([os.path.join(REF, "libggml_ref.so"), G.BACKEND_LIB, os.path.join(REF, "libgpt2_ref.so")])
    cpu = lib.ggml_backend_cpu_init()
    lib.ggml_backend_cpu_set_n_threads(cpu, min(16, os.cpu_count() or 1))
    gpu = lib.ggml_backend_mi355x_init(0) if max(layers) > 0 else None
    assert gpu or max(layers) == 0, "ggml_backend_mi355x_init failed"
    prompt = "Once upon a time the cat sat on the mat and the dog"
    for spec in specs:
        parts = spec.split(":")
        ngl = int(parts[0])
        flags = int(parts[1]) if len(parts) > 1 else 0
        in_buft = lib.ggml_backend_mi355x_host_buffer_type() if len(parts) > 2 and parts[2] == "h" else None
        arr = (G.c_void_p * 2)(gpu, cpu) if ngl > 0 else (G.c_void_p * 1)(cpu)
        m = lib.gpt2_model_load_sched_ex(model_path.encode(), arr, 2 if ngl > 0 else 1, ngl, 1024, 8, flags, in_buft)
        assert m, "gpt2_model_load_sched failed"
        splits = lib.gpt2_sched_n_splits(m)
        wrap = gpt2.Model.__new__(gpt2.Model)
        wrap.lib, wrap.m, wrap.n_vocab = lib, m, 50257
        toks = wrap.tokenize(prompt)
        outs, n_past = [], 0
        for i in range(0, len(toks), 8):
            outs.append(wrap.eval(n_past, toks[i:i + 8], all_logits=True))
            n_past += len(toks[i:i + 8])
        nxt = int(np.argmax(outs[-1][-1]))
        for _ in range(8):
            lg = wrap.eval(n_past, [nxt])
            outs.append(lg)
            n_past += 1
            nxt = int(np.argmax(lg[-1]))
        splits = max(splits, lib.gpt2_sched_n_splits(m))
        np.save(os.path.join(out_dir, "ngl" + spec.replace(":", "_") + ".npy"), np.concatenate(outs))
        print(f"n_gpu_layers={spec}: splits={splits}")
        lib.gpt2_model_free(m)
        wrap.m = None
    if gpu:
        lib.ggml_backend_free(gpu)
    lib.ggml_backend_free(cpu)


if __name__ == "__main__":
    main()
