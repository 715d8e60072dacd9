#!/usr/bin/env python3
"""Benchmark of the MI355X ggml backend on BASELINE.json's headline metric.

Workload (BASELINE.json metric "Q4_K 4096x4096 mul_mat GB/s-effective", configs[1..2] shape):
  one step = one ggml_backend_graph_compute of a graph holding R independent GGML_OP_MUL_MAT
  nodes  Y_r = W_r . X_r  with W_r Q4_K [K=4096, N=4096] (R distinct weight copies, >256 MiB in
  total so the 256 MiB Infinity Cache cannot serve them) and X_r f32 [4096, B=1] -- i.e. R
  decode-style GEMVs, inputs resident in HBM, activation quantization included.
  value = R * algorithmic bytes * steps * world / max-over-ranks wall time of the timed steps,
  algorithmic bytes per unit = N*(K/256)*144 + 4*K*B + 4*N*B.

Multi-GPU (--gpus N via torch.distributed.run): independent prompts shard across GPUs, each
rank owns a full replica of its weights and runs the same per-GPU work ("scaling": "weak"); the
only collective is the timing barrier / max-reduction (no data-path exchange exists).

Extra fields: "roofline" (dominant kernel: algorithmic bytes per launch / HIP-event duration on
the backend's own stream, vs 8 TB/s HBM), "cpu_baseline" (the reference ggml CPU backend,
oracle/_ref/libggml_ref.so, timed on this host -- rank 0, N=1 only) and a per-config sweep.
"""
from __future__ import annotations

import argparse
import ctypes
import glob
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "ggml-imax_amd"))

from ggml_mi355x import ggml as G  # noqa: E402
from ggml_mi355x import synth  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s HBM3E (spec)
MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: ~2.5 PF dense f16/bf16 MFMA
I8_PEAK_TOPS = 2 * MFMA_PEAK_TFLOPS  # MI355X_MICROARCH.md, Matrix cores: I8 32x32x32 runs at 2x the BF16 rate per clock
TYPE_NAMES = {"q4_K": 12, "q5_K": 13, "q4_0": 2, "q8_0": 8, "f16": 1}


def unit_bytes(t: int, K: int, N: int, B: int) -> int:
    return G.row_size(t, K) * N + 4 * K * B + 4 * N * B


class MulMatWorkload:
    """R independent mul_mat nodes in one graph, all tensors resident on `backend`."""

    def __init__(self, lib, backend, t, K, N, B, R, seed=42):
        self.lib, self.backend, self.t, self.K, self.N, self.B, self.R = lib, backend, t, K, N, B, R
        ovh = lib.ggml_tensor_overhead() * (3 * R + 8) + lib.ggml_graph_overhead_custom(4 * R + 16, False)
        self.ctx = G.Context(lib, ovh, no_alloc=True)
        c = self.ctx.ctx
        self.w = [lib.ggml_new_tensor_2d(c, t, K, N) for _ in range(R)]
        self.x = [lib.ggml_new_tensor_2d(c, G.GGML_TYPE_F32, K, B) for _ in range(R)]
        self.y = [lib.ggml_mul_mat(c, self.w[r], self.x[r]) for r in range(R)]
        self.graph = lib.ggml_new_graph_custom(c, 4 * R + 16, False)
        for y in self.y:
            lib.ggml_build_forward_expand(self.graph, y)
        self.buf = lib.ggml_backend_alloc_ctx_tensors(c, backend)
        assert self.buf, "device allocation failed"
        wf = synth.uniform(seed, K * N)
        wq = np.empty(G.row_size(t, K) * N, np.uint8)
        lib.ggml_quantize_chunk(t, wf.ctypes.data, wq.ctypes.data, 0, N, K, None)
        self.wq = wq
        for r in range(R):
            G.tensor_set(lib, self.w[r], wq)
            G.tensor_set(lib, self.x[r], synth.uniform(seed + 1 + r, K * B))

    def step(self):
        st = self.lib.ggml_backend_graph_compute_async(self.backend, self.graph)
        assert st == 0, st

    def free(self):
        self.lib.ggml_backend_buffer_free(self.buf)
        self.ctx.free()


def host_cpus():
    """CPUs this process may run on: the affinity mask, capped by the cgroup CPU quota (on the GPU
    box the mask lists the whole machine, the quota is this job's share), plus the host topology."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = max(1, int(int(q) // int(period)))
    except (OSError, ValueError):
        pass
    model, cores, sockets = "unknown", None, set()
    try:
        for line in open("/proc/cpuinfo"):
            k, _, v = line.partition(":")
            k, v = k.strip(), v.strip()
            if k == "model name":
                model = v
            elif k == "cpu cores":
                cores = int(v)
            elif k == "physical id":
                sockets.add(v)
    except OSError:
        pass
    usable = min(aff, quota) if quota else aff
    return {"threads": int(os.environ.get("BENCH_CPU_THREADS", usable)), "affinity_cpus": aff, "cgroup_quota_cpus": quota,
            "model": model, "physical_cores_per_socket": cores, "sockets": len(sockets) or None,
            "logical_cpus": os.cpu_count()}


def cpu_baseline(t, K, N, B, seconds=10.0):
    """The reference ggml CPU backend (oracle/_ref/libggml_ref.so, compiled from the reference
    sources with its own x86 flags) on a bounded sample of the same workload, with one thread per
    CPU this job may use (host_cpus)."""
    ref_path = os.path.join(REPO, "oracle", "_ref", "libggml_ref.so")
    if not os.path.exists(ref_path):
        return None
    ref = G.Lib([ref_path], isolated=True)
    hc = host_cpus()
    threads = hc["threads"]
    cpu = ref.ggml_backend_cpu_init()
    ref.ggml_backend_cpu_set_n_threads(cpu, threads)
    R = 32  # same rotation depth as the GPU run: the weights do not fit the CPU caches either
    wl = MulMatWorkload(ref, cpu, t, K, N, B, R)
    wl.lib.ggml_backend_graph_compute(cpu, wl.graph)  # warm-up
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        ref.ggml_backend_graph_compute(cpu, wl.graph)
        n += 1
    dt = time.perf_counter() - t0
    wl.free()
    ref.ggml_backend_free(cpu)
    units = n * R
    return {
        "value": round(units * unit_bytes(t, K, N, B) / dt / 1e9, 2), "unit": "GB/s",
        "cores": threads, "kind": "reference",
        "sample": f"{units} mul_mats ({n} graphs x {R}) of the same workload in {dt:.1f} s; "
                  f"us/mul_mat={dt / units * 1e6:.1f}",
        "host": hc,
    }


GPT2_PROMPT = "Once upon a time the cat sat on the mat and the dog ran away from the big red house"


def gpt2_bench(lib, backend, n_decode=128, n_batch=8, path=None, label="GPT-2-117M f16 (synthetic seeded weights, 239.08 MB)",
               parity="teacher-forced logits within 7e-4 of max|logit| of the reference CPU (<= 1e-3, tests/test_gpt2.py)"):
    """BASELINE config 4: GPT-2-117M f16 (synthetic seeded weights, legacy ggml file) on MI355X.
    Prompt in n_batch chunks, then n_decode greedy single-token steps, logits read back each step
    (as examples/gpt-2/main-backend.cpp's gpt2_eval does). Returns decode tokens/s and the
    reference program's ms/token definition (predict time / n_past, prompt tokens included)."""
    from ggml_mi355x import gpt2
    path = path or gpt2.ensure_model()
    m = gpt2.Model(lib, path, backend, n_ctx=1024, n_batch=n_batch)
    try:
        toks = m.tokenize(GPT2_PROMPT)
        n_past, t_pred = 0, 0.0
        t0 = time.perf_counter()
        for i in range(0, len(toks), n_batch):
            lg = m.eval(n_past, toks[i:i + n_batch])
            n_past += len(toks[i:i + n_batch])
        t_prompt = time.perf_counter() - t0
        nxt = int(np.argmax(lg[-1]))
        # decode steps read the last token's logits in place (the host staging the logits are
        # copied into behind each graph, gpt2_logits_host) instead of a copy per step
        for _ in range(8):  # warm-up decode steps (not timed), then restart the context
            lg = m.eval(n_past, [nxt], copy=False)
            nxt = int(np.argmax(lg[-1]))
        n_past = len(toks)
        t_eval = 0.0  # gpt2_eval alone: the reference program's "predict time" (sampling excluded)
        t0 = time.perf_counter()
        for _ in range(n_decode):
            te = time.perf_counter()
            lg = m.eval(n_past, [nxt], copy=False)
            t_eval += time.perf_counter() - te
            n_past += 1
            nxt = int(np.argmax(lg[-1]))
        t_dec = time.perf_counter() - t0
        st = m.stats()
        gs = None
        if hasattr(lib, "ggml_backend_mi355x_graph_stats"):
            import ctypes
            arr = (ctypes.c_int64 * 4)()
            lib.ggml_backend_mi355x_graph_stats(backend, arr)
            gs = {"captured_plans": arr[0], "instantiations": arr[1], "in_place_updates": arr[2], "direct_computes": arr[3]}
        t_pred = t_prompt + t_dec
        return {"model": label, "decode_tokens_per_s": round(n_decode / t_dec, 1),
                "ms_per_decode_token": round(t_dec / n_decode * 1e3, 4),
                # main-backend.cpp:880 / :936 time gpt2_eval (logits readback included) apart from the
                # host sampling (:897-901, its own "sample time"); ms_per_decode_token above includes
                # this harness's host argmax
                "ms_per_decode_token_predict": round(t_eval / n_decode * 1e3, 4),
                "prompt_tokens": len(toks), "prompt_tokens_per_s": round(len(toks) / t_prompt, 1),
                "ms_per_token_reference_definition": round(t_pred / n_past * 1e3, 4),
                "graph_nodes": st["nodes"], "kernel_launches_per_token": lib.ggml_backend_mi355x_last_launch_count(backend),
                "host_us_per_token": {k: st[k] for k in ("us_build", "us_alloc", "us_inputs", "us_launch", "us_prebuild", "us_wait",
                                                         "us_readback") if k in st},
                "graphs": gs, "parity": parity}
    finally:
        m.free()


def gpt2_f16_bench(lib, backend, n_decode):
    """Config 4 headline: default (tree-order, fast) decode kernels, logits within 1e-3 of the
    reference CPU; beside it mmv_order=1 (the reference's summation order), logits bit-identical."""
    r = gpt2_bench(lib, backend, n_decode)
    lib.ggml_backend_mi355x_set_tuning(b"mmv_order", 1)
    try:
        ex = gpt2_bench(lib, backend, n_decode, parity="decode-path logits bit-identical to the reference CPU (tests/test_gpt2.py)")
    finally:
        lib.ggml_backend_mi355x_set_tuning(b"mmv_order", -1)
    r["mmv_order_1"] = {k: ex[k] for k in ("decode_tokens_per_s", "ms_per_decode_token", "parity")}
    return r


def gpt2_q4k_bench(lib, backend, n_decode):
    """The same decode loop on the model quantized to Q4_K by gpt2.quantize_model (byte-identical
    to examples/gpt-2/quantize.cpp), with the backend's default settings: a graph whose quantized
    mul_mats consume computed activations runs its decode reductions in the reference CPU's order
    (mmv_order -1 = auto), so the logits are bit-identical to the reference's
    (tests/test_gpt2.py) and meet the 1e-3 logit bar; the tree-order mode (mmv_order=0) is reported
    beside it with its measured deviation (it does NOT meet 1e-3 on this model)."""
    from ggml_mi355x import gpt2
    path = gpt2.ensure_quantized_model(lib, "q4_k")
    r = gpt2_bench(lib, backend, n_decode, path=path, label="GPT-2-117M Q4_K (quantize.cpp q4_k of the synthetic model), default settings",
                   parity="logits bit-identical to the reference CPU at every teacher-forced step (max |d| = 0 <= 1e-3)")
    lib.ggml_backend_mi355x_set_tuning(b"mmv_order", 0)
    try:
        tree = gpt2_bench(lib, backend, n_decode, path=path, label="same, mmv_order=0 (tree-order GEMV)",
                          parity="NOT within 1e-3: 1.4-2.1e-2 of max|logit| (the model re-quantizes activations every layer)")
    finally:
        lib.ggml_backend_mi355x_set_tuning(b"mmv_order", -1)
    r["tree_order"] = {k: tree[k] for k in ("decode_tokens_per_s", "ms_per_decode_token", "parity")}
    return r


def gpt2_batched_bench(lib, backend, n_parallel=8, n_steps=48):
    """examples/gpt-2/main-batched.cpp's workload on MI355X: an 8-token prompt decoded once and
    shared by n_parallel sequences (KV cells + seq ids), then n_steps batches of one greedy token per
    sequence through the KQ-mask graph (ggml_backend_graph_compute: captured into hipGraphs inside
    graph_compute). Aggregate decode tokens/s over all sequences; the same loop with graph capture
    off beside it (graph_compute decode with and without capture)."""
    from ggml_mi355x import gpt2
    # KV cells: the prompt once + one per sequence and step (main-batched.cpp's n_kv_req)
    n_ctx = 8 + (4 + n_steps) * n_parallel
    m = gpt2.Model(lib, gpt2.ensure_model(), backend, n_ctx=(n_ctx + 255) // 256 * 256, n_batch=8)

    def run():
        prompt = m.tokenize(GPT2_PROMPT)[:8]
        m.kv_clear()
        lg = m.decode_batch(prompt, list(range(len(prompt))), [0] * len(prompt), all_logits=False)
        for s in range(1, n_parallel):
            m.kv_seq_cp(0, s, -1, -1)
        nxt = [int(np.argmax(lg[-1]))] * n_parallel
        seqs = list(range(n_parallel))
        for w in range(4):  # warm-up steps (not timed)
            lg = m.decode_batch(nxt, [len(prompt) + w] * n_parallel, seqs)
            nxt = [int(v) for v in np.argmax(lg, axis=1)]
        t0 = time.perf_counter()
        t_dec = 0.0  # gpt2_decode alone: main-batched.cpp's "predict time" (:1171-1180), sampling excluded
        for t in range(n_steps):
            # (logits read in place from the pinned staging, as main-batched.cpp reads llama's
            # logits buffer; copy=True adds a 1.6 MB host memcpy per step)
            td = time.perf_counter()
            lg = m.decode_batch(nxt, [len(prompt) + 4 + t] * n_parallel, seqs, copy=False)
            t_dec += time.perf_counter() - td
            nxt = [int(v) for v in np.argmax(lg, axis=1)]
        predict.append(t_dec)
        return time.perf_counter() - t0

    def stats():
        a = (ctypes.c_int64 * 6)()
        lib.ggml_backend_mi355x_graph_stats_ex(backend, a, 6)
        return list(a)

    def bstats():
        a = (ctypes.c_int64 * 2)()
        if hasattr(lib, "gpt2_batch_stats"):
            lib.gpt2_batch_stats(m.m, a)
        return list(a)

    predict = []
    try:
        run()  # untimed pass: first captures of each topology, allocator and cache warm-up
        s0, b0 = stats(), bstats()
        dt = run()
        dt_pred = predict[-1]
        s1, b1 = stats(), bstats()
        r = {"workload": f"{n_parallel} sequences sharing an 8-token prompt, {n_steps} batched decode steps (main-batched.cpp)",
             "decode_tokens_per_s": round(n_parallel * n_steps / dt, 1), "ms_per_step": round(dt / n_steps * 1e3, 4),
             "ms_per_step_predict": round(dt_pred / n_steps * 1e3, 4),
             "note": "ms_per_step: the whole step incl. this harness's host argmax over the 8 x n_vocab logits; "
                     "ms_per_step_predict: gpt2_decode alone, main-batched.cpp's predict time (its sampling is timed apart)",
             "kernel_launches_per_step": lib.ggml_backend_mi355x_last_launch_count(backend),
             "parity": "within 1e-3 of the reference CPU, bit-identical with mmv_order=1 (tests/test_gpt2.py batched tests)",
             "graph_compute_calls": {"direct": s1[3] - s0[3], "replays": s1[4] - s0[4], "captures": s1[5] - s0[5]},
             "steps": {"prebuilt_plan_launches": b1[0] - b0[0], "built_on_the_spot": b1[1] - b0[1],
                       "note": "a step's graph is built, allocated and captured as a plan while the device runs the previous "
                               "step; its inputs (tokens, positions, KQ mask) go in as one async copy"}}
        if hasattr(lib, "ggml_backend_mi355x_set_graph_capture"):
            lib.ggml_backend_mi355x_set_graph_capture(backend, False)
            try:
                dt2 = run()
            finally:
                lib.ggml_backend_mi355x_set_graph_capture(backend, True)
            r["no_graph_capture"] = {"decode_tokens_per_s": round(n_parallel * n_steps / dt2, 1), "ms_per_step": round(dt2 / n_steps * 1e3, 4)}
        return r
    finally:
        m.free()


def gpt2_cpu_baseline(threads, n_predict=64, path=None):
    """The reference's own examples/gpt-2/main-backend.cpp (oracle/_ref/gpt-2-backend, built from
    the reference sources) on the same synthetic model, CPU backend: its printed ms per token."""
    import re
    import subprocess
    exe = os.path.join(REPO, "oracle", "_ref", "gpt-2-backend")
    if not os.path.exists(exe):
        return None
    from ggml_mi355x import gpt2
    p = subprocess.run([exe, "-m", path or gpt2.ensure_model(), "-p", GPT2_PROMPT, "-n", str(n_predict), "-s", "1", "-t", str(threads)],
                       capture_output=True, text=True, timeout=600)
    mt = re.search(r"predict time =\s*([\d.]+) ms /\s*([\d.]+) ms per token", p.stdout)
    if p.returncode != 0 or not mt:
        return None
    ms_tok = float(mt.group(2))
    return {"value": round(1e3 / ms_tok, 1), "unit": "tokens/s", "ms_per_token": ms_tok, "cores": threads, "kind": "reference",
            "sample": f"examples/gpt-2/main-backend.cpp (reference program) -n {n_predict} -t {threads}: predict time / n_past"}


def shard_range(total: int, world: int, rank: int):
    """Balanced contiguous shard [start, start+count) of `total` units for `rank` (prompt columns
    of a batched mul_mat: each GPU runs its columns against its own weight replica)."""
    base, rem = divmod(total, world)
    start = rank * base + min(rank, rem)
    return start, base + (1 if rank < rem else 0)


def row_shard(N: int, world: int, rank: int, rounding: int = 64):
    """Rows [r0, r1) of an N-row weight held by `rank` on the tensor-split row path: cumulative
    equal fractions rounded down to the GEMM's 64-row tile, the last rank takes the rest (the
    split of ggml_backend_mi355x_split_buffer_type / ggml-cuda.cu:660-676)."""
    def start(r):
        if r == 0:
            return 0
        v = (N * r) // world
        return v - v % rounding
    return start(rank), (N if rank == world - 1 else start(rank + 1))


def reassemble_rows(y_all: np.ndarray, N: int, world: int, B: int) -> np.ndarray:
    """Y [B, N] from the all-gathered row slices: y_all holds, per rank, a [B, rows_max] block
    (ggml dst layout: rows contiguous per column), of which the first r1 - r0 rows are real."""
    rows_max = y_all.size // (world * B)
    blocks = y_all.reshape(world, B, rows_max)
    out = np.empty((B, N), y_all.dtype)
    for r in range(world):
        r0, r1 = row_shard(N, world, r)
        out[:, r0:r1] = blocks[r, :, :r1 - r0]
    return out


class _DevArray:
    """__cuda_array_interface__ over a device pointer (ggml device buffer memory -> torch view)."""

    def __init__(self, ptr: int, n: int, typestr: str = "<f4"):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": typestr, "data": (ptr, False), "version": 2, "strides": None}


def torch_view(torch, lib, t, device):
    """A torch f32 view of ggml tensor `t`'s device memory (no copy)."""
    n = int(lib.ggml_nelements(t))
    return torch.as_tensor(_DevArray(G.tensor_data_ptr(lib, t), n), device=device)


def torch_bytes(torch, lib, t, device):
    """A torch uint8 view of ggml tensor `t`'s device bytes (quantized tensors)."""
    return torch.as_tensor(_DevArray(G.tensor_data_ptr(lib, t), int(lib.ggml_nbytes(t)), "|u1"), device=device)


def rowsplit_prefill(lib, backend, dist, world, rank, device, torch, steps=5, K=4096, N=4096, B=512, return_y=False):
    """Optional tensor-split row path over RCCL (north_star "RCCL only for
    the optional tensor-split row path"): rank r holds rows row_shard(N) of one Q4_K weight; per
    step rank 0 quantizes its prompt activations X (f32 [K, B]) ONCE on its GPU to Q8_K rows (the
    weight's vec_dot type: a GGML_OP_CPY F32 -> Q8_K graph) and broadcasts those bytes to every rank
    (RCCL over xGMI; 292 B per 256 values instead of 1 KB -- as the reference ships src1 quantized
    once, ggml-cuda.cu:1551-1565); each rank computes its Y rows from them (MUL_MAT with a Q8_K
    src1, read as it lies) and the row slices are all-gathered (RCCL)."""
    r0, r1 = row_shard(N, world, rank)
    rows = r1 - r0
    rows_max = max(row_shard(N, world, r)[1] - row_shard(N, world, r)[0] for r in range(world))
    ovh = lib.ggml_tensor_overhead() * 8 + 2 * lib.ggml_graph_overhead()
    ctx = G.Context(lib, ovh, no_alloc=True)
    c = ctx.ctx
    w = lib.ggml_new_tensor_2d(c, 12, K, rows)
    x = lib.ggml_new_tensor_2d(c, G.GGML_TYPE_F32, K, B)
    xq = lib.ggml_new_tensor_2d(c, 15, K, B)  # GGML_TYPE_Q8_K
    y = lib.ggml_mul_mat(c, w, xq)
    ypad = lib.ggml_new_tensor_2d(c, G.GGML_TYPE_F32, rows_max, B)  # all_gather needs equal slices
    gq = lib.ggml_new_graph(c)
    lib.ggml_build_forward_expand(gq, lib.ggml_cpy(c, x, xq))
    g = lib.ggml_new_graph(c)
    lib.ggml_build_forward_expand(g, y)
    buf = lib.ggml_backend_alloc_ctx_tensors(c, backend)
    wf = synth.uniform(42, K * N)[r0 * K:r1 * K]
    wq = np.empty(G.row_size(12, K) * rows, np.uint8)
    lib.ggml_quantize_chunk(12, wf.ctypes.data, wq.ctypes.data, 0, rows, K, None)
    G.tensor_set(lib, w, wq)
    if rank == 0:
        G.tensor_set(lib, x, synth.uniform(43, K * B))
    xq_t = torch_bytes(torch, lib, xq, device)
    y_t = torch_view(torch, lib, y, device).view(B, rows)
    ypad_t = torch_view(torch, lib, ypad, device).view(B, rows_max)
    y_all = torch.empty(world * B * rows_max, dtype=torch.float32, device=device)

    def step():
        if rank == 0:
            lib.ggml_backend_graph_compute(backend, gq)
            lib.ggml_backend_synchronize(backend)  # the quants are written before RCCL reads them
        dist.broadcast(xq_t, src=0)
        torch.cuda.current_stream().synchronize()  # Xq landed before the backend stream reads it
        lib.ggml_backend_graph_compute(backend, g)
        if rows != rows_max:
            ypad_t[:, :rows].copy_(y_t)
            dist.all_gather_into_tensor(y_all, ypad_t.reshape(-1))
        else:
            dist.all_gather_into_tensor(y_all, y_t.reshape(-1))

    step()  # warm-up (RCCL communicator set-up)

    def run():
        for _ in range(steps):
            step()

    def sync():
        lib.ggml_backend_synchronize(backend)
        torch.cuda.synchronize()

    dt = timed_region(run, sync, dist, device)
    y_full = reassemble_rows(y_all.cpu().numpy(), N, world, B)
    res = {"workload": f"Q4_K {K}x{N} x B={B}, rows split over {world} ranks: X quantized to Q8_K once on rank 0, RCCL broadcast "
                       f"of the {int(lib.ggml_nbytes(xq))} quant bytes, local GEMM, RCCL all-gather of Y",
           "rows_per_rank": rows, "TFLOP/s": round(2.0 * K * N * B * steps / dt / 1e12, 2),
           "us_per_step": round(dt / steps * 1e6, 2)}
    res.update(rowsplit_parity(y_full, K, N, B))
    lib.ggml_backend_buffer_free(buf)
    ctx.free()
    return (res, y_full) if return_y else res


def rowsplit_parity(y_full, K, N, B):
    """Element-wise check of the reassembled Y [B, N] against the reference's own output for this
    exact workload (tests/golden: BASELINE config 5, weights splitmix64 seed 42 quantized to Q4_K,
    X seed 43; every 16th column from the reference CPU build, plus the SHA-256 of its whole Y)."""
    gold = os.path.join(REPO, "tests", "golden")
    try:
        man = {c["name"]: c for c in json.load(open(os.path.join(gold, "manifest.json")))["cases"]}
        c = man[f"P_q4_K_{K}x{N}_b{B}"]
        ys = np.fromfile(os.path.join(gold, c["name"] + ".ys.f32"), dtype=np.float32).reshape(-1, N)
    except (OSError, KeyError, ValueError):
        return {"parity": "no golden fixture for this shape"}
    got = y_full[::c["y_col_step"]]
    err = float(np.max(np.abs(got.astype(np.float64) - ys)) / np.max(np.abs(ys)))
    return {"max_rel_err_vs_reference": err, "parity_ok": err <= 1e-5,
            "parity": f"every {c['y_col_step']}th column ({got.shape[0]} x {N}) element-wise vs the reference CPU output (<= 1e-5)"}


def timed_region(run, sync, dist=None, device=None):
    """Barrier + sync on both sides of `run()`; returns the MAX wall time over ranks."""
    sync()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    run()
    sync()
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    if dist:
        import torch
        t = torch.tensor([dt], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    return dt


def event_time_per_step(torch, wl, stream_ptr, iters=20):
    """HIP-event duration of one step on the backend's own stream (ms)."""
    s = torch.cuda.ExternalStream(stream_ptr)
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(iters):
        wl.step()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / iters


def load_traffic(kernel_prefix: str):
    """Per-launch HBM bytes of the dominant kernel from the newest committed PMC summary
    (tools/pmc_traffic.py -> profiles/*_pmc_traffic.json): (bytes, source file, kernel name), or
    (None, None, None). Not measured in this run: rocprofv3 counters need their own process."""
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "*pmc_traffic*.json")))
    for f in reversed(files):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        for k, v in d.get("kernels", {}).items():
            if k.startswith(kernel_prefix):
                return v.get("hbm_bytes_per_launch"), os.path.relpath(f, REPO), k
    return None, None, None


class RotatedSingle:
    """ONE mul_mat per graph (the shape a dependent decode layer presents): R graphs over R weight
    copies, computed round-robin, so every launch streams a weight the caches do not hold."""

    def __init__(self, lib, backend, t, K, N, B, R):
        self.wls = [MulMatWorkload(lib, backend, t, K, N, B, 1, seed=42) for _ in range(R)]
        self.i = 0

    def step(self):
        self.wls[self.i].step()
        self.i = (self.i + 1) % len(self.wls)

    def free(self):
        for w in self.wls:
            w.free()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--type", default="q4_K", choices=sorted(TYPE_NAMES))
    ap.add_argument("--K", type=int, default=4096)
    ap.add_argument("--N", type=int, default=4096)
    ap.add_argument("--B", type=int, default=1)
    ap.add_argument("--rotate", type=int, default=32)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-sweep", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-gpt2", action="store_true")
    ap.add_argument("--gpt2-tokens", type=int, default=128)
    args = ap.parse_args()

    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # BENCH_DIST_BACKEND: the collective backend ("nccl" = RCCL, the default; "gloo" rehearses the
    # multi-rank path with ranks sharing a GPU -- tests/test_bench_gpu.py runs 2 ranks on one device)
    dist_backend = os.environ.get("BENCH_DIST_BACKEND", "nccl")
    ndev = torch.cuda.device_count() if dist_backend == "gloo" else 0
    device_index = local_rank % ndev if ndev else local_rank
    dist = None
    coll_device = None  # where the timing collective's tensor lives (gloo: host)
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(device_index)
        if dist_backend == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", device_index))
            coll_device = torch.device("cuda", device_index)

    lib = G.runtime()
    backend = G.mi355x_backend(lib, device_index)
    stream_ptr = lib.ggml_backend_mi355x_get_stream(backend)
    t = TYPE_NAMES[args.type]
    K, N, B, R = args.K, args.N, args.B, args.rotate
    wl = MulMatWorkload(lib, backend, t, K, N, B, R)

    for _ in range(args.warmup):
        wl.step()

    def sync():
        lib.ggml_backend_synchronize(backend)
        torch.cuda.synchronize()

    # HIP events on the backend's own stream bracket exactly the timed steps
    ext_stream = torch.cuda.ExternalStream(stream_ptr)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)

    def run_steps():
        ev0.record(ext_stream)
        for _ in range(args.steps):
            wl.step()
        ev1.record(ext_stream)

    dt = timed_region(run_steps, sync, dist, coll_device)

    ub = unit_bytes(t, K, N, B)
    value = R * ub * args.steps * world / dt / 1e9
    launches = lib.ggml_backend_mi355x_last_launch_count(backend)

    # dominant kernel: HIP events on the backend's own stream around the timed steps. The
    # backend serves the R independent mul_mats of a step with `launches` kernel launches (1 when
    # the fused streaming GEMV groups them), so per launch: bytes = R*ub/launches, duration =
    # step time / launches.
    ev1.synchronize()
    step_ms = ev0.elapsed_time(ev1) / args.steps
    launches = max(launches, 1)
    bytes_per_launch = R * ub / launches
    achieved = bytes_per_launch / (step_ms / 1e3 / launches) / 1e9
    traffic, traffic_src, traffic_kernel = load_traffic("void (anonymous namespace)::k_mmv_stream<(anonymous namespace)::FmtKQ<false>")

    result = {
        "metric": "Q4_K 4096x4096 mul_mat GB/s-effective (+ GPT-2 tokens/s), 1 GPU",
        "value": round(value, 2),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "q4_K x q8_K int8-dot, f32 accumulate" if t in (12, 13) else args.type,
        "data": "synthetic (splitmix64 seed 42 weights quantized by the runtime's ggml_quantize_chunk; seeded X)",
        "config": {"workload": f"{R} independent {args.type} {K}x{N} mul_mat (GEMV, B={B}) per step, rotated weights "
                               f"({R * G.row_size(t, K) * N / 2**20:.0f} MiB)", "K": K, "N": N, "B": B,
                   "rotated_copies": R, "parallelism": f"replica x{world}"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "traffic_source": {"file": traffic_src, "kernel": traffic_kernel,
                                        "note": "PMC FETCH_SIZE/WRITE_SIZE passes of the same bench command, committed profile; not this run"},
                     "kernel_launches_per_step": launches, "event_ms_per_step": round(step_ms, 4),
                     "algorithmic_bytes_per_launch": int(bytes_per_launch),
                     "note": "achieved = algorithmic bytes per launch (R mul_mats x (N*K/256*144 + 4K + 4N) / launches) "
                             "/ HIP-event duration per launch on the backend stream over the timed steps; activation quantization is inside "
                             "the kernel; traffic = PMC HBM bytes per launch (tools/pmc_traffic.py, gfx950-corrected)"},
    }

    if rank == 0 and world == 1 and not args.no_sweep:
        sweep = {}
        for name, tt, k, n in (("q4_0_4096x4096", 2, 4096, 4096), ("q4_K_4096x11008", 12, 4096, 11008),
                               ("q5_K_4096x11008", 13, 4096, 11008), ("q8_0_4096x11008", 8, 4096, 11008)):
            r = max(8, int(320 * 2**20 // (G.row_size(tt, k) * n)) + 1)
            w2 = MulMatWorkload(lib, backend, tt, k, n, 1, r)
            for _ in range(3):
                w2.step()
            lib.ggml_backend_synchronize(backend)
            ms = event_time_per_step(torch, w2, stream_ptr, iters=10)
            sweep[name] = {"GB/s": round(r * unit_bytes(tt, k, n, 1) / (ms / 1e3) / 1e9, 1),
                           "us_per_mul_mat": round(ms * 1e3 / r, 2)}
            w2.free()
        # one Q4_K 4096^2 GEMV per graph (no grouping), 32 rotated weights
        w1 = RotatedSingle(lib, backend, 12, 4096, 4096, 1, 32)
        for _ in range(64):
            w1.step()
        lib.ggml_backend_synchronize(backend)
        ms = event_time_per_step(torch, w1, stream_ptr, iters=256)
        sweep["q4_K_4096x4096_single_graph"] = {
            "GB/s": round(unit_bytes(12, 4096, 4096, 1) / (ms / 1e3) / 1e9, 1), "us_per_mul_mat": round(ms * 1e3, 2),
            "launches_per_graph": lib.ggml_backend_mi355x_last_launch_count(backend),
            "note": "one mul_mat per graph_compute, 32 weight copies round-robin; HIP events over 256 graphs"}
        w1.free()
        # configs[4]: batched prefill Q4_K 4096x4096 on MFMA tiles (per GPU; the 8-GPU run shards
        # the 512 prompt columns, 64 per GPU), plus the mid-batch sizes. 32 rotated weight copies
        # (288 MiB, more than the 256 MB Infinity Cache): R independent mul_mats per graph (grouped
        # launches), and the same mul_mat alone in its own graph (a dependent layer's shape)
        RP = 32
        for bb in (512, 64, 32, 16):
            w3 = MulMatWorkload(lib, backend, 12, 4096, 4096, bb, RP)
            for _ in range(3):
                w3.step()
            lib.ggml_backend_synchronize(backend)
            ms = event_time_per_step(torch, w3, stream_ptr, iters=10)
            flops = 2.0 * 4096 * 4096 * bb * RP
            us = ms * 1e3 / RP
            flops_per = flops / RP
            e = {"TFLOP/s": round(flops / (ms / 1e3) / 1e12, 2), "us_per_mul_mat": round(us, 2),
                 "GB/s_effective": round(unit_bytes(12, 4096, 4096, bb) / (us / 1e6) / 1e9, 1),
                 "launches_per_mul_mat": lib.ggml_backend_mi355x_last_launch_count(backend) / RP, "rotated_copies": RP}
            w3.free()
            w4 = RotatedSingle(lib, backend, 12, 4096, 4096, bb, RP)
            for _ in range(2 * RP):
                w4.step()
            lib.ggml_backend_synchronize(backend)
            ms1 = event_time_per_step(torch, w4, stream_ptr, iters=4 * RP)
            e["us_per_mul_mat_one_per_graph"] = round(ms1 * 1e3, 2)
            w4.free()
            if bb == 512:
                peak = I8_PEAK_TOPS / 2  # Q4_K: two int8 weight planes per weight (mmq_exact.hip)
                e["roofline"] = {"bound": "mfma", "achieved": round(flops_per / (us / 1e6) / 1e12, 2), "peak": peak,
                                 "unit": "TFLOP/s", "frac": round(flops_per / (us / 1e6) / 1e12 / peak, 4),
                                 "note": "useful 2*N*K*B / HIP-event time of the whole mul_mat (activation quantizer + GEMM) vs "
                                         "the dense I8 MFMA peak (5 POP/s) / 2: the exact block sums run as two "
                                         "v_mfma_i32_32x32x32_i8 per 32-deep K step (Q4_K weight planes q*(sc bit field))"}
            elif bb == 64:
                e["roofline"] = {"bound": "hbm", "achieved": e["GB/s_effective"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                 "frac": round(e["GB/s_effective"] / HBM_PEAK_GBS, 4),
                                 "note": "algorithmic bytes (weights + f32 activations + f32 outputs) / HIP-event time of the "
                                         "whole mul_mat (activation quantizer + GEMM)"}
            sweep[f"q4_K_4096x4096_b{bb}_prefill"] = e
        result["sweep"] = sweep

    if world > 1 and not args.no_sweep:
        # BASELINE config 5: ONE B=512 prefill (Q4_K 4096x4096) prompt-sharded across the GPUs --
        # each rank runs its columns against its own weight replica; no data-path collective
        start, cnt = shard_range(512, world, rank)
        w4 = MulMatWorkload(lib, backend, 12, 4096, 4096, cnt, 8)
        for _ in range(3):
            w4.step()

        def run_pf():
            for _ in range(5):
                w4.step()

        dtp = timed_region(run_pf, sync, dist, coll_device)
        result["prefill_sharded"] = {"workload": "8 x Q4_K 4096x4096 x B=512 per step, columns sharded over ranks",
                                     "columns_per_rank": cnt, "TFLOP/s": round(2.0 * 4096 * 4096 * 512 * 8 * 5 / dtp / 1e12, 2),
                                     "us_per_mul_mat": round(dtp / 5 / 8 * 1e6, 2)}
        w4.free()

    if world > 1 and not args.no_sweep:
        # the optional tensor-split row path (RCCL): reported beside the main line, never fatal to it
        try:
            if dist_backend != "nccl":
                raise RuntimeError(f"the row-split leg exchanges device tensors over RCCL; collective backend is {dist_backend}")
            result["prefill_rowsplit_rccl"] = rowsplit_prefill(lib, backend, dist, world, rank, coll_device, torch)
        except Exception as e:  # noqa: BLE001
            result["prefill_rowsplit_rccl"] = {"error": f"{type(e).__name__}: {e}"}

    if rank == 0 and world == 1 and not args.no_gpt2:
        # BASELINE config 4 (the metric's "+ GPT-2 tokens/s" half)
        result["gpt2"] = gpt2_f16_bench(lib, backend, args.gpt2_tokens)
        result["gpt2_q4_k"] = gpt2_q4k_bench(lib, backend, args.gpt2_tokens)
        try:  # an auxiliary line: its failure must not take the headline with it
            result["gpt2_batched"] = gpt2_batched_bench(lib, backend)
        except Exception as e:  # noqa: BLE001
            result["gpt2_batched"] = {"error": f"{type(e).__name__}: {e}"}

    if rank == 0 and world == 1 and not args.no_cpu:
        result["cpu_baseline"] = cpu_baseline(t, K, N, B, args.cpu_seconds)
        threads = host_cpus()["threads"]
        if "gpt2" in result:
            result["gpt2"]["cpu_baseline"] = gpt2_cpu_baseline(threads)
        if "gpt2_q4_k" in result:
            from ggml_mi355x import gpt2
            result["gpt2_q4_k"]["cpu_baseline"] = gpt2_cpu_baseline(threads, path=gpt2.ensure_quantized_model(lib, "q4_k"))

    wl.free()
    lib.ggml_backend_free(backend)
    if rank == 0:
        print(json.dumps(result))
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
