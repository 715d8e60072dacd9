#!/usr/bin/env python3
"""Regenerate tests/golden/ from the real reference build (dev container only).

1. `make -C oracle ref` compiles /root/reference/src/*.c into oracle/_ref/libggml_ref.so and
   links oracle/gen_fixtures.c against it.
2. gen_fixtures writes the reference's outputs (quantized weights, dequantized weights,
   quantized activations, CPU mul_mat outputs) for seeded splitmix64 inputs.
3. Small blobs are copied here; for the BASELINE.json-sized cases only the SHA-256 of the
   reference-quantized weights and the full output vectors are kept (weights are regenerated
   from their seeds by ggml_mi355x.synth + a quantizer and checked against the hash).

The reference itself never travels to the GPU box; these data files do.
"""
from __future__ import annotations

import hashlib
import json
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))


def main() -> int:
    subprocess.check_call(["make", "-C", os.path.join(REPO, "oracle"), "ref", "-j8"])
    gen = os.path.join(REPO, "oracle", "_ref", "gen_fixtures")
    with tempfile.TemporaryDirectory() as tmp:
        subprocess.check_call([gen, tmp])
        cases = json.load(open(os.path.join(tmp, "cases.json")))
        for c in cases:
            wq = os.path.join(tmp, c["name"] + ".wq.bin")
            c["wq_sha256"] = hashlib.sha256(open(wq, "rb").read()).hexdigest()
            c["wq_bytes"] = os.path.getsize(wq)
            if c["name"].startswith("P_"):
                # prefill-sized outputs: SHA-256 of the whole Y [B][N] plus every step-th column
                y = np.fromfile(os.path.join(tmp, c["name"] + ".y.f32"), np.float32).reshape(c["B"], c["N"])
                c["y_sha256"] = hashlib.sha256(y.tobytes()).hexdigest()
                c["y_col_step"] = step = max(1, c["B"] // 32)
                np.ascontiguousarray(y[::step]).tofile(os.path.join(HERE, c["name"] + ".ys.f32"))
        for fn in sorted(os.listdir(tmp)):
            if fn == "cases.json":
                continue
            if fn.startswith(("L_", "P_")) and fn.endswith(".wq.bin"):
                continue  # large weights: hash only
            if fn.startswith("P_") and fn.endswith(".y.f32"):
                continue  # hash + sampled columns only
            shutil.copy(os.path.join(tmp, fn), os.path.join(HERE, fn))
        manifest = {
            "generator": "oracle/gen_fixtures.c linked to oracle/_ref/libggml_ref.so",
            "reference": "NAIST-Archlab/ggml-imax @ v2 (/root/reference), gcc -O3 -mavx -mavx2 -mfma -mf16c -msse3",
            "rng": "splitmix64, value=(u>>40)*2^-24*2-1; W[n*K+k] from wseed, X[b*K+k] from xseed",
            "cases": cases,
        }
        with open(os.path.join(HERE, "manifest.json"), "w") as f:
            json.dump(manifest, f, indent=1)
    print(f"wrote {len(cases)} cases to {HERE}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
