"""Multi-process path of bench.py on CPU (gloo, world_size 2) -- SURVEY.md section 8e.

The path shards without a data-path collective: independent prompts / prompt columns go to
different ranks, each with its own weight replica. These tests run bench.py's own helpers
(shard_range, timed_region) under torch.distributed with the gloo backend, with the reference
CPU backend (oracle/_ref/libggml_ref.so, test infrastructure) computing each rank's shard of a
Q4_K mul_mat: the column shards gathered from the ranks must equal the unsharded product bit for
bit, and the reported time must be the maximum over ranks.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import REPO

import bench
from ggml_mi355x import ggml as G

REF_LIB = os.path.join(REPO, "oracle", "_ref", "libggml_ref.so")


def test_shard_range_covers_exactly():
    for total in (1, 7, 64, 512, 513):
        for world in (1, 2, 3, 8):
            seen = []
            for r in range(world):
                s, c = bench.shard_range(total, world, r)
                seen.extend(range(s, s + c))
            assert seen == list(range(total))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, K, N, B, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ref = G.Lib([REF_LIB], isolated=True)
        cpu = ref.ggml_backend_cpu_init()
        ref.ggml_backend_cpu_set_n_threads(cpu, 2)
        start, cnt = bench.shard_range(B, world, rank)
        # every rank builds the same weights (seeded) and the full activation matrix; it keeps
        # only its columns, as a prompt-sharded prefill does
        full = bench.MulMatWorkload(ref, cpu, 12, K, N, B, 1, seed=5)
        x_all = G.tensor_get(ref, full.x[0]).reshape(B, K)
        mine = bench.MulMatWorkload(ref, cpu, 12, K, N, cnt, 1, seed=5)
        G.tensor_set(ref, mine.x[0], x_all[start:start + cnt])

        def run():
            ref.ggml_backend_graph_compute(cpu, mine.graph)

        dt = bench.timed_region(run, lambda: None, dist, None)
        y = G.tensor_get(ref, mine.y[0]).reshape(cnt, N)
        # gather the shards (test only: the product path has no collective)
        gathered = [None] * world
        dist.all_gather_object(gathered, y)
        if rank == 0:
            ref.ggml_backend_graph_compute(cpu, full.graph)
            y_full = G.tensor_get(ref, full.y[0]).reshape(B, N)
            np.save(os.path.join(out_dir, "full.npy"), y_full)
            np.save(os.path.join(out_dir, "sharded.npy"), np.concatenate(gathered))
        t_local = torch.tensor([dt], dtype=torch.float64)
        np.save(os.path.join(out_dir, f"dt{rank}.npy"), t_local.numpy())
        mine.free()
        full.free()
        ref.ggml_backend_free(cpu)
    finally:
        dist.destroy_process_group()


@pytest.mark.skipif(not os.path.exists(REF_LIB), reason="make -C oracle ref")
@pytest.mark.parametrize("B", [8, 9])
def test_prompt_sharded_mul_mat_gloo(tmp_path, B):
    K, N, world = 512, 96, 2
    mp.spawn(_worker, args=(world, _free_port(), K, N, B, str(tmp_path)), nprocs=world, join=True)
    full = np.load(tmp_path / "full.npy")
    sharded = np.load(tmp_path / "sharded.npy")
    assert sharded.shape == full.shape
    assert np.array_equal(sharded.view(np.uint32), full.view(np.uint32))
    dts = [float(np.load(tmp_path / f"dt{r}.npy")[0]) for r in range(world)]
    assert dts[0] == dts[1] > 0  # every rank reports the max over ranks


# ------------------------------------------------------------------ tensor-split row path (RCCL leg)

def test_row_shard_covers_exactly():
    for N in (64, 1000, 4096, 11008):
        for world in (1, 2, 3, 8):
            seen = []
            for r in range(world):
                r0, r1 = bench.row_shard(N, world, r)
                assert r0 % 64 == 0
                seen.extend(range(r0, r1))
            assert seen == list(range(N))


def _rowsplit_worker(rank, world, port, K, N, B, out_dir):
    """bench.rowsplit_prefill's exchange on gloo: rank 0 quantizes X to Q8_K rows (the weight's
    vec_dot type) and broadcasts the bytes, each rank computes its rows of W.Xq with the reference
    CPU backend (MUL_MAT reads a Q8_K src1 as it lies), all-gather the padded row slices,
    reassemble."""
    from ggml_mi355x import synth
    Q8_K = 15
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ref = G.Lib([REF_LIB], isolated=True)
        cpu = ref.ggml_backend_cpu_init()
        ref.ggml_backend_cpu_set_n_threads(cpu, 2)
        with G.Context(ref, 1024, no_alloc=True):
            pass  # ggml_init: the fp16 tables ggml_quantize_chunk's rounding reads
        r0, r1 = bench.row_shard(N, world, rank)
        rows = r1 - r0
        rows_max = max(bench.row_shard(N, world, r)[1] - bench.row_shard(N, world, r)[0] for r in range(world))
        x = synth.uniform(43, K * B)
        nq = K // 256 * 292 * B
        if rank == 0:  # X -> Q8_K rows on the reference CPU (GGML_OP_CPY: quantize_row_q8_K)
            ovh = ref.ggml_tensor_overhead() * 4 + ref.ggml_graph_overhead()
            with G.Context(ref, ovh, no_alloc=True) as c:
                xt = ref.ggml_new_tensor_2d(c.ctx, G.GGML_TYPE_F32, K, B)
                q = ref.ggml_cpy(c.ctx, xt, ref.ggml_new_tensor_2d(c.ctx, Q8_K, K, B))
                g = ref.ggml_new_graph(c.ctx)
                ref.ggml_build_forward_expand(g, q)
                buf = ref.ggml_backend_alloc_ctx_tensors(c.ctx, cpu)
                G.tensor_set(ref, xt, x)
                ref.ggml_backend_graph_compute(cpu, g)
                xq = torch.from_numpy(G.tensor_get(ref, q, np.uint8).copy())
                ref.ggml_backend_buffer_free(buf)
        else:
            xq = torch.zeros(nq, dtype=torch.uint8)
        dist.broadcast(xq, src=0)
        wf = synth.uniform(42, K * N)
        wq = np.empty(G.row_size(12, K) * rows, np.uint8)
        ref.ggml_quantize_chunk(12, wf[r0 * K:r1 * K].ctypes.data, wq.ctypes.data, 0, rows, K, None)

        def build(c):
            wt = ref.ggml_new_tensor_2d(c, 12, K, rows)
            xt = ref.ggml_new_tensor_2d(c, Q8_K, K, B)
            return [(wt, wq), (xt, xq.numpy())], ref.ggml_mul_mat(c, wt, xt)

        y = G.graph_once(ref, cpu, build).reshape(B, rows)
        ypad = np.zeros((B, rows_max), np.float32)
        ypad[:, :rows] = y
        y_all = torch.empty(world * B * rows_max)
        dist.all_gather_into_tensor(y_all, torch.from_numpy(ypad).reshape(-1))
        if rank == 0:
            np.save(os.path.join(out_dir, "rowsplit.npy"), bench.reassemble_rows(y_all.numpy(), N, world, B))
            full = bench.MulMatWorkload(ref, cpu, 12, K, N, B, 1, seed=5)
            wq_full = np.empty(G.row_size(12, K) * N, np.uint8)
            ref.ggml_quantize_chunk(12, wf.ctypes.data, wq_full.ctypes.data, 0, N, K, None)
            G.tensor_set(ref, full.w[0], wq_full)
            G.tensor_set(ref, full.x[0], x)
            ref.ggml_backend_graph_compute(cpu, full.graph)
            np.save(os.path.join(out_dir, "full.npy"), G.tensor_get(ref, full.y[0]).reshape(B, N))
            full.free()
        ref.ggml_backend_free(cpu)
    finally:
        dist.destroy_process_group()


@pytest.mark.skipif(not os.path.exists(REF_LIB), reason="make -C oracle ref")
@pytest.mark.parametrize("world,N", [(2, 512), (3, 320)])
def test_rowsplit_exchange_gloo(tmp_path, world, N):
    K, B = 512, 4
    mp.spawn(_rowsplit_worker, args=(world, _free_port(), K, N, B, str(tmp_path)), nprocs=world, join=True)
    full = np.load(tmp_path / "full.npy")
    split = np.load(tmp_path / "rowsplit.npy")
    assert np.array_equal(split.view(np.uint32), full.view(np.uint32))
