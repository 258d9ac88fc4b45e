"""Multi-rank row sharding + all-gather of C, on CPU with gloo, world_size 2
and 3: the host side of the multi-rank path (the library's row split, lamm_hip_shard_rows,
and the slab interleave) with each rank's slab computed by the oracle -- no GPU here; the
gathered C must equal the single-process result bit for bit (the same per-row arithmetic on
both sides).  The HIP slabs and the library's RCCL all-gather path are covered on the GPU by
tests/test_gpu_shard.py and bench.py's multi-GPU self-check."""
import os
import socket
import sys

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "la-llama.cpp_amd"))
from lamm_amd.shard import gather_rows, row_shard  # noqa: E402


def test_row_shard_covers_all_rows():
    for M in (1, 7, 64, 70, 4096, 4097):
        for world in (1, 2, 3, 8):
            for align in (1, 16, 256):
                spans = [row_shard(M, world, r, align) for r in range(world)]
                assert spans[0][0] == 0 and spans[-1][1] == M
                for (a0, a1), (b0, b1) in zip(spans, spans[1:]):
                    assert a1 == b0 and a0 <= a1
                for a0, a1 in spans[:-1]:
                    assert a0 % align == 0 or a0 == M
    # the reference's job_size = M / nth drops M % nth rows; we do not
    assert row_shard(67, 3, 2) == (45, 67)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, M, N, K, align, q):
    sys.path.insert(0, HERE)
    import oracle_lib as ol

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        o = ol.Oracle()
        rng = np.random.default_rng(5)
        a = rng.standard_normal((M, K), dtype=np.float32)
        b = rng.standard_normal((N, K), dtype=np.float32)
        A = o.quantize(ol.Q4_0, a).reshape(M, -1)
        B = o.quantize(ol.Q8_0, b, ol.QUANT_AVX)
        r0, r1 = row_shard(M, world, rank, align)
        c = o.mul_mat(ol.Q4_0, r1 - r0, N, K, np.ascontiguousarray(A[r0:r1]), B) if r1 > r0 \
            else np.zeros((N, 0), np.float32)
        full = gather_rows(dist, torch.from_numpy(np.ascontiguousarray(c, dtype=np.float32)), M, N, world, rank, align)
        if rank == 0:
            q.put(full.numpy().copy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,M,align", [(2, 70, 16), (3, 67, 1), (2, 256, 128)])
def test_gather_rows_gloo(world, M, align):
    import oracle_lib as ol

    N, K = 9, 512
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, M, N, K, align, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    o = ol.Oracle()
    rng = np.random.default_rng(5)
    a = rng.standard_normal((M, K), dtype=np.float32)
    b = rng.standard_normal((N, K), dtype=np.float32)
    want = o.mul_mat(ol.Q4_0, M, N, K, o.quantize(ol.Q4_0, a), o.quantize(ol.Q8_0, b, ol.QUANT_AVX))
    np.testing.assert_array_equal(got, want.reshape(N, M))
