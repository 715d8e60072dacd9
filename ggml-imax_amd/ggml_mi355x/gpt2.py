"""GPT-2 (BASELINE config 4): synthetic GPT-2-117M model files and a wrapper over include/gpt2-mi355x.h.

No GPT-2 weights exist offline (the reference's download scripts need network), so models are
synthetic and seeded, written in the legacy ggml format that examples/gpt-2/main-backend.cpp:101-439
loads -- the layout examples/gpt-2/convert-ckpt-to-ggml.py:91-151 produces: magic, 6 int32 hparams,
vocab (len + bytes), then per tensor (n_dims, name length, ftype, ne[0..], name, data), with "model/wte"
and every ".../w" matrix in f16 and everything else f32. At 117M shapes the file holds 239.08 MB of
tensor data, the figure the reference prints for the real model.
"""
from __future__ import annotations

import ctypes
import os
import struct

import numpy as np

from . import ggml as G

GPT2_117M = dict(n_vocab=50257, n_ctx=1024, n_embd=768, n_head=12, n_layer=12)
EOT = 50256


class gpt2_hparams_c(ctypes.Structure):
    _fields_ = [("n_vocab", ctypes.c_int32), ("n_ctx", ctypes.c_int32), ("n_embd", ctypes.c_int32),
                ("n_head", ctypes.c_int32), ("n_layer", ctypes.c_int32), ("ftype", ctypes.c_int32),
                ("eps", ctypes.c_float)]


def synthetic_vocab(n_vocab: int, seed: int = 0) -> list[bytes]:
    """Deterministic GPT-2-like vocabulary: printable bytes, ' '+char, then syllable words with and
    without a leading space; the last id is <|endoftext|>."""
    rng = np.random.default_rng(seed)
    toks: list[bytes] = []
    seen = set()

    def add(t: bytes):
        if t not in seen and len(toks) < n_vocab - 1:
            seen.add(t)
            toks.append(t)

    for c in range(32, 127):
        add(bytes([c]))
    add(b"\n")
    for c in b"abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789":
        add(b" " + bytes([c]))
    cons = [b"b", b"c", b"d", b"f", b"g", b"h", b"k", b"l", b"m", b"n", b"p", b"r", b"s", b"t", b"v", b"w",
            b"th", b"st", b"ch", b"sh", b"tr", b"pl"]
    vows = [b"a", b"e", b"i", b"o", b"u", b"ea", b"ou", b"y"]
    while len(toks) < n_vocab - 1:
        ns = int(rng.integers(1, 4))
        w = b"".join(cons[int(rng.integers(len(cons)))] + vows[int(rng.integers(len(vows)))] for _ in range(ns))
        if rng.random() < 0.3:
            w += cons[int(rng.integers(len(cons)))]
        add((b" " + w) if rng.random() < 0.6 else w)
    toks.append(b"<|endoftext|>")
    return toks


def write_synthetic_model(path: str, seed: int = 117, ftype: int = 1, **hp) -> str:
    """Write a seeded GPT-2 model (default 117M shapes) in the legacy ggml format; returns path.

    Init follows GPT-2's: N(0, 0.02) matrices and embeddings, residual projections scaled by
    1/sqrt(2*n_layer), layer norms near (1, 0), small biases.
    """
    h = dict(GPT2_117M)
    h.update(hp)
    E, L, V, C = h["n_embd"], h["n_layer"], h["n_vocab"], h["n_ctx"]
    rng = np.random.default_rng(seed)
    vocab = synthetic_vocab(V, seed)
    tmp = path + ".tmp"
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(tmp, "wb") as f:
        f.write(struct.pack("i", 0x67676D6C))
        for k in ("n_vocab", "n_ctx", "n_embd", "n_head", "n_layer"):
            f.write(struct.pack("i", h[k]))
        f.write(struct.pack("i", ftype))
        f.write(struct.pack("i", V))
        for t in vocab:
            f.write(struct.pack("i", len(t)))
            f.write(t)

        def tensor(name: str, data: np.ndarray):
            is_mat = name == "model/wte" or name.endswith("/w")
            cur = ftype if is_mat else 0
            arr = data.astype(np.float16 if cur == 1 else np.float32)
            nm = name.encode()
            f.write(struct.pack("iii", arr.ndim, len(nm), cur))
            for i in range(arr.ndim):
                f.write(struct.pack("i", arr.shape[arr.ndim - 1 - i]))
            f.write(nm)
            arr.tofile(f)

        def normal(shape, std):
            return (rng.standard_normal(shape, dtype=np.float32) * np.float32(std))

        tensor("model/wte", normal((V, E), 0.02))
        tensor("model/wpe", normal((C, E), 0.01))
        proj_std = 0.02 / np.sqrt(2 * L)
        for i in range(L):
            p = f"model/h{i}"
            tensor(p + "/ln_1/g", 1.0 + normal((E,), 0.05))
            tensor(p + "/ln_1/b", normal((E,), 0.02))
            tensor(p + "/attn/c_attn/w", normal((3 * E, E), 0.02))
            tensor(p + "/attn/c_attn/b", normal((3 * E,), 0.02))
            tensor(p + "/attn/c_proj/w", normal((E, E), proj_std))
            tensor(p + "/attn/c_proj/b", normal((E,), 0.02))
            tensor(p + "/ln_2/g", 1.0 + normal((E,), 0.05))
            tensor(p + "/ln_2/b", normal((E,), 0.02))
            tensor(p + "/mlp/c_fc/w", normal((4 * E, E), 0.02))
            tensor(p + "/mlp/c_fc/b", normal((4 * E,), 0.02))
            tensor(p + "/mlp/c_proj/w", normal((E, 4 * E), proj_std))
            tensor(p + "/mlp/c_proj/b", normal((E,), 0.02))
        tensor("model/ln_f/g", 1.0 + normal((E,), 0.05))
        tensor("model/ln_f/b", normal((E,), 0.02))
    os.replace(tmp, path)
    return path


def default_model_path() -> str:
    root = os.environ.get("GRAFT_REPO_ROOT") or os.path.dirname(G.PKG_ROOT)
    return os.path.join(root, "models", "gpt2-117M-synth-f16.bin")


def ensure_model(path: str | None = None, seed: int = 117) -> str:
    path = path or default_model_path()
    if not os.path.exists(path):
        write_synthetic_model(path, seed=seed)
    return path


# examples/gpt-2/quantize.cpp:114-128 (tensors quantized); names as common-ggml.cpp:6-17 spells them
QUANT_TENSORS = [r"model/wte", r"model/lm_head", r"model/h.*/attn/c_attn/w", r"model/h.*/attn/c_proj/w",
                 r"model/h.*/mlp/c_fc/w", r"model/h.*/mlp/c_proj/w"]
FTYPES = {"q4_0": (2, G.GGML_TYPE_Q4_0), "q8_0": (7, G.GGML_TYPE_Q8_0), "q4_k": (12, G.GGML_TYPE_Q4_K),
          "q5_k": (13, G.GGML_TYPE_Q5_K)}
GGML_QNT_VERSION, GGML_QNT_VERSION_FACTOR = 2, 1000


def quantize_model(lib: G.Lib, src: str, dst: str, qtype: str) -> str:
    """The reference's examples/gpt-2/quantize.cpp on a legacy GPT-2 file (common-ggml.cpp:19-236
    ggml_common_quantize_0): the header's ftype becomes the target (+ GGML_QNT_VERSION * 1000), the
    2-D tensors named in QUANT_TENSORS are converted to f32 and quantized row by row with
    ggml_quantize_chunk (imatrix = NULL), everything else is copied."""
    import re
    ftype, ttype_q = FTYPES[qtype.lower()]
    pats = [re.compile(p) for p in QUANT_TENSORS]
    tmp = dst + ".tmp"
    os.makedirs(os.path.dirname(os.path.abspath(dst)), exist_ok=True)
    with open(src, "rb") as fi, open(tmp, "wb") as fo:
        hdr = struct.unpack("7i", fi.read(28))  # magic, n_vocab, n_ctx, n_embd, n_head, n_layer, ftype
        fo.write(struct.pack("7i", *hdr[:6], ftype + GGML_QNT_VERSION * GGML_QNT_VERSION_FACTOR))
        n_vocab = struct.unpack("i", fi.read(4))[0]
        fo.write(struct.pack("i", n_vocab))
        for _ in range(n_vocab):
            (ln,) = struct.unpack("i", fi.read(4))
            fo.write(struct.pack("i", ln))
            fo.write(fi.read(ln))
        while True:
            head = fi.read(12)
            if len(head) < 12:
                break
            n_dims, name_len, ttype = struct.unpack("3i", head)
            ne = list(struct.unpack(f"{n_dims}i", fi.read(4 * n_dims)))
            name = fi.read(name_len)
            nel = int(np.prod(ne))
            quant = n_dims == 2 and any(p.fullmatch(name.decode()) for p in pats)
            if quant:
                assert ttype in (0, 1), f"{name!r}: cannot quantize type {ttype}"
                data = np.fromfile(fi, dtype=np.float16 if ttype == 1 else np.float32, count=nel).astype(np.float32)
                out = np.empty(G.row_size(ttype_q, ne[0]) * (nel // ne[0]), np.uint8)
                lib.ggml_quantize_chunk(ttype_q, data.ctypes.data, out.ctypes.data, 0, nel // ne[0], ne[0], None)
                ttype = ttype_q
            else:
                out = np.fromfile(fi, dtype=np.uint8, count=nel * (4 if ttype == 0 else 2))
            fo.write(struct.pack("3i", n_dims, name_len, ttype))
            fo.write(struct.pack(f"{n_dims}i", *ne))
            fo.write(name)
            out.tofile(fo)
    os.replace(tmp, dst)
    return dst


def ensure_quantized_model(lib: G.Lib, qtype: str, path: str | None = None) -> str:
    base = ensure_model()
    path = path or base.replace("-f16.bin", f"-{qtype.lower()}.bin")
    if not os.path.exists(path):
        quantize_model(lib, base, path, qtype)
    return path


class Model:
    """One loaded GPT-2 on a backend (gpt2_model_load); eval() returns logits as numpy."""

    def __init__(self, lib: G.Lib, path: str, backend, n_ctx: int = 0, n_batch: int = 8, host_io: bool = True):
        """host_io: on an MI355X backend, token ids / positions in pinned host memory read by the
        device in place and the logits staged through it (gpt2_model_load_ex)."""
        if not lib.has("gpt2_model_load"):
            raise RuntimeError("this library set has no GPT-2 driver (lib/libgpt2_mi355x.so)")
        self.lib = lib
        self.backend = backend
        if host_io and lib.has("gpt2_model_load_ex") and lib.has("ggml_backend_is_mi355x") and lib.ggml_backend_is_mi355x(backend):
            self.m = lib.gpt2_model_load_ex(path.encode(), backend, n_ctx, n_batch, lib.ggml_backend_mi355x_host_buffer_type())
        else:
            self.m = lib.gpt2_model_load(path.encode(), backend, n_ctx, n_batch)
        if not self.m:
            raise RuntimeError(f"gpt2_model_load({path}) failed")
        hp = gpt2_hparams_c()
        lib.gpt2_model_hparams(self.m, ctypes.byref(hp))
        self.hp = hp
        self.n_vocab = hp.n_vocab
        # the host staging of the last token's logits (host_io), read in place by eval(copy=False)
        self._staged = None
        # (the staging holds min(n_ctx, n_batch) rows of logits, gpt2_model_load_ex)
        self._staged_bytes = hp.n_vocab * min(hp.n_ctx, n_batch if n_batch > 0 else 8) * 4
        if lib.has("gpt2_logits_host"):
            ptr = lib.gpt2_logits_host(self.m)
            if ptr:
                self._staged = np.ctypeslib.as_array((ctypes.c_float * hp.n_vocab).from_address(ptr)).reshape(1, hp.n_vocab)
        self._tok = np.zeros(1, dtype=np.int32)

    def eval(self, n_past: int, tokens, all_logits: bool = False, copy: bool = True) -> np.ndarray:
        """copy=False (last token's logits, host_io models): a view of the host staging, valid
        until the next eval."""
        if not copy and not all_logits and self._staged is not None and len(tokens) == 1:
            self._tok[0] = tokens[0]
            if self.lib.gpt2_eval(self.m, n_past, self._tok.ctypes.data, 1, None, 0) != 0:
                raise RuntimeError("gpt2_eval failed")
            return self._staged
        tok = np.ascontiguousarray(np.asarray(tokens, dtype=np.int32))
        n = len(tok)
        out = np.empty((n if all_logits else 1, self.n_vocab), dtype=np.float32)
        rc = self.lib.gpt2_eval(self.m, n_past, tok.ctypes.data, n, out.ctypes.data, 1 if all_logits else 0)
        if rc != 0:
            raise RuntimeError("gpt2_eval failed")
        return out

    def decode_batch(self, tokens, pos, seq_id, all_logits: bool = True, copy: bool = True) -> np.ndarray:
        """gpt2_decode_batch (examples/gpt-2/main-batched.cpp gpt2_decode): token i of sequence
        seq_id[i] at position pos[i]; logits [n_tokens or 1, n_vocab]. copy=False (host_io models):
        a view of the pinned logits staging, valid until the next eval / decode_batch (as
        llama_get_logits_ith returns a pointer into the context's logits)."""
        tok = np.ascontiguousarray(np.asarray(tokens, dtype=np.int32))
        p = np.ascontiguousarray(np.asarray(pos, dtype=np.int32))
        s = np.ascontiguousarray(np.asarray(seq_id, dtype=np.int32))
        n = len(tok)
        assert len(p) == n and len(s) == n
        rows = n if all_logits else 1
        view = None
        if not copy and self._staged is not None and self.lib.has("gpt2_logits_host"):
            ptr = self.lib.gpt2_logits_host(self.m)
            if ptr and rows * self.n_vocab * 4 <= self._staged_bytes:
                view = np.ctypeslib.as_array((ctypes.c_float * (rows * self.n_vocab)).from_address(ptr)).reshape(rows, self.n_vocab)
        out = view if view is not None else np.empty((rows, self.n_vocab), dtype=np.float32)
        rc = self.lib.gpt2_decode_batch(self.m, n, tok.ctypes.data, p.ctypes.data, s.ctypes.data,
                                        None if view is not None else out.ctypes.data, 1 if all_logits else 0)
        if rc != 0:
            raise RuntimeError(f"gpt2_decode_batch failed ({rc})")
        return out

    def kv_seq_cp(self, src: int, dst: int, p0: int = -1, p1: int = -1):
        self.lib.gpt2_kv_cache_seq_cp(self.m, src, dst, p0, p1)

    def kv_clear(self):
        self.lib.gpt2_kv_cache_clear(self.m)

    def stats(self) -> dict:
        n = ctypes.c_int()
        b, a, i, c = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        self.lib.gpt2_last_eval_stats(self.m, ctypes.byref(n), ctypes.byref(b), ctypes.byref(a), ctypes.byref(i), ctypes.byref(c))
        r = {"nodes": n.value, "us_build": b.value, "us_alloc": a.value, "us_inputs": i.value, "us_compute": c.value}
        if hasattr(self.lib, "gpt2_last_eval_timing"):
            t = (ctypes.c_int64 * 4)()
            self.lib.gpt2_last_eval_timing(self.m, t)
            r.update(us_launch=t[0], us_prebuild=t[1], us_wait=t[2], us_readback=t[3])
        return r

    def tokenize(self, text: str) -> list[int]:
        buf = np.empty(4096, dtype=np.int32)
        n = self.lib.gpt2_tokenize(self.m, text.encode(), buf.ctypes.data, len(buf))
        return buf[:min(n, len(buf))].tolist()

    def token_text(self, i: int) -> bytes:
        return self.lib.gpt2_token_text(self.m, i)

    @property
    def weight_bytes(self) -> int:
        return self.lib.gpt2_model_size(self.m)

    def free(self):
        if self.m:
            self.lib.gpt2_model_free(self.m)
            self.m = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def run_batched(model: "Model", prompt: list[int], n_parallel: int, forced: list[list[int]], copy: bool = True) -> np.ndarray:
    """main-batched.cpp's flow, teacher-forced: the prompt decoded once as sequence 0, its cells
    shared with sequences 1..n_parallel-1 (gpt2_kv_cache_seq_cp), then one batch per step holding
    token forced[t][s] of every sequence s at position len(prompt) + t. Returns the prompt's last
    logits followed by every step's n_parallel rows: [1 + steps * n_parallel, n_vocab].
    copy=False: each step's logits read in place from the staging (decode_batch), saved by value here."""
    model.kv_clear()
    n = len(prompt)
    outs = [np.array(model.decode_batch(prompt, list(range(n)), [0] * n, all_logits=False, copy=copy))]
    for s in range(1, n_parallel):
        model.kv_seq_cp(0, s, -1, -1)
    for t, row in enumerate(forced):
        assert len(row) == n_parallel
        outs.append(np.array(model.decode_batch(row, [n + t] * n_parallel, list(range(n_parallel)), all_logits=True, copy=copy)))
    return np.concatenate(outs)
