"""Multi-GPU row sharding on the HIP path, rehearsed on one device: a loopback
communicator (lamm_hip_comm_init_all with one device listed `world` times -- RCCL refuses
duplicate devices, so the ranks exchange slabs by device copies) runs exactly the pack /
unshard kernels and slab bookkeeping the RCCL path runs.  Each rank computes its slab of C
with the HIP kernels (A's rows [r0, r0 + rows), lamm_hip_shard_rows); after the all-gather
every rank's C must equal the slabs bit for bit and the oracle within the parity tolerance.
The ncclAllGather itself runs in bench.py's multi-GPU mode (one process per GPU), which checks
the gathered C against a single-GPU computation of the same rows."""
import numpy as np
import pytest

from conftest import rel_err
import oracle_lib as ol

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
import lamm_amd as la  # noqa: E402

ORACLE = ol.Oracle()
TOL = 1e-3


def _case(t, M, N, K, seed):
    rng = np.random.default_rng(seed)
    A_q = ORACLE.quantize(t, rng.standard_normal((M, K), dtype=np.float32))
    vt = la.vec_dot_type(t)
    B_q = ORACLE.quantize(vt, rng.standard_normal((N, K), dtype=np.float32),
                          ol.QUANT_AVX if vt in (ol.Q8_0, ol.Q8_1) else ol.QUANT_REF)
    return A_q, B_q


CASES = [(ol.Q4_0, 4096, 1, 4096), (ol.Q4_0, 1000, 1, 512), (ol.Q4_0, 4096, 64, 1024), (ol.Q8_0, 777, 9, 512),
         (ol.Q4_K, 513, 3, 512), (ol.F16, 300, 20, 256)]


@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("case", CASES, ids=[f"{ol.NAMES[c[0]]}-{c[1]}x{c[2]}x{c[3]}" for c in CASES])
def test_sharded_hip_slabs_gathered(world, case):
    t, M, N, K = case
    align = 16
    if t in ol.KQ_TYPES:
        A_q = ol.random_kq_blocks(t, M, K, np.random.default_rng(7))
        B_q = ORACLE.quantize(ol.Q8_K, np.random.default_rng(8).standard_normal((N, K), dtype=np.float32))
    else:
        A_q, B_q = _case(t, M, N, K, seed=M + N + world)
    kb, bpb = K // la.blck_size(t), la.type_size(t)
    lda = kb
    while (lda * bpb) % 16:
        lda += 1
    Ap = np.zeros((M, lda * bpb), np.uint8)
    Ap[:, :kb * bpb] = A_q.reshape(M, kb * bpb)
    A = torch.from_numpy(np.concatenate([Ap.reshape(-1), np.zeros(64, np.uint8)])).cuda()
    B = torch.from_numpy(B_q.copy()).cuda()
    comm = la.Comm.all([0] * world)
    assert comm.size == world and comm.local_ranks == world
    stream = torch.cuda.current_stream().cuda_stream
    slabs, Cs = [], []
    for r in range(world):
        r0, rows = la.shard_rows(M, world, r, align)
        slab = torch.full((max(rows, 1) * N,), float("nan"), dtype=torch.float32, device="cuda")
        if rows:
            la.mul_mat_torch(t, A[r0 * lda * bpb:], B, slab, rows, N, K, lda=lda, ldc=rows)
        slabs.append(slab)
        Cs.append(torch.full((N * M,), float("nan"), dtype=torch.float32, device="cuda"))
    rows_of = [la.shard_rows(M, world, r, align)[1] for r in range(world)]
    comm.allgather_rows([s.data_ptr() for s in slabs], [max(n, 1) for n in rows_of], [c.data_ptr() for c in Cs], M, M,
                        N, align, [stream] * world)
    torch.cuda.synchronize()
    want = np.concatenate([slabs[r].cpu().numpy()[:rows_of[r] * N].reshape(N, rows_of[r]) for r in range(world)], axis=1)
    ref = ORACLE.mul_mat(t, M, N, K, A_q, B_q)
    Ad = ORACLE.dequantize(t, A_q, M, K).astype(np.float64)
    Bd = ORACLE.dequantize(la.vec_dot_type(t), B_q, N, K).astype(np.float64)
    absdot = np.abs(Bd) @ np.abs(Ad).T
    for r in range(world):
        got = Cs[r].cpu().numpy().reshape(N, M)
        np.testing.assert_array_equal(got, want)
        assert rel_err(got, ref, absdot).max() < TOL
    comm.close()


def _slabs_and_gather(comm, locals_, t, M, N, K, devices, streams, seed):
    """every local rank computes its slab on its device/stream, then one all-gather"""
    align = 16
    world = comm.size
    A_q, B_q = _case(t, M, N, K, seed=seed)
    kb, bpb = K // la.blck_size(t), la.type_size(t)
    slabs, Cs, lds = [], [], []
    for i, g in enumerate(locals_):
        with torch.cuda.device(devices[i]):
            A = torch.from_numpy(np.concatenate([A_q, np.zeros(64, np.uint8)])).cuda()
            B = torch.from_numpy(B_q.copy()).cuda()
            r0, rows = la.shard_rows(M, world, g, align)
            slab = torch.full((max(rows, 1) * N,), float("nan"), dtype=torch.float32, device="cuda")
            if rows:
                la.mul_mat_torch(t, A[r0 * kb * bpb:], B, slab, rows, N, K, ldc=rows, stream=streams[i].cuda_stream)
            slabs.append(slab)
            lds.append(max(rows, 1))
            Cs.append(torch.full((N * M,), float("nan"), dtype=torch.float32, device="cuda"))
    comm.allgather_rows([s.data_ptr() for s in slabs], lds, [c.data_ptr() for c in Cs], M, M, N, align,
                        [s.cuda_stream for s in streams])
    for i in range(len(locals_)):
        with torch.cuda.device(devices[i]):
            torch.cuda.synchronize()
    ref = ORACLE.mul_mat(t, M, N, K, A_q, B_q)
    return [c.cpu().numpy().reshape(N, M) for c in Cs], ref


@pytest.mark.parametrize("N", [1, 5])
def test_loopback_gather_separate_streams(N):
    """The loopback exchange with one stream per rank (its copies are ordered by events only, so
    it can be graph-captured): repeated calls reusing the same C buffers stay bit-exact."""
    world, t, M, K = 3, ol.Q4_0, 1000, 512
    comm = la.Comm.all([0] * world)
    streams = [torch.cuda.Stream() for _ in range(world)]
    first = None
    for rep in range(3):
        Cs, ref = _slabs_and_gather(comm, list(range(world)), t, M, N, K, [0] * world, streams, seed=11)
        for c in Cs:
            np.testing.assert_array_equal(c, Cs[0])
            assert np.isfinite(c).all()
        first = Cs[0] if first is None else first
        np.testing.assert_array_equal(Cs[0], first)
    comm.close()


def test_rccl_one_rank_allgather():
    """The RCCL path itself on a one-GPU box: a one-rank communicator (lamm_hip_comm_init_rank,
    ncclAllGather in place) -- the call sequence every rank of a multi-GPU job makes."""
    comm = la.Comm.rank(1, 0, la.comm_unique_id(), 0)
    Cs, ref = _slabs_and_gather(comm, [0], ol.Q4_0, 512, 3, 512, [0], [torch.cuda.Stream()], seed=12)
    assert np.isfinite(Cs[0]).all() and np.abs(Cs[0] - ref).max() <= 1e-3 * np.abs(ref).max()
    comm.close()


@pytest.mark.skipif(not torch.cuda.is_available() or torch.cuda.device_count() < 2, reason="needs >= 2 GPUs")
def test_rccl_allgather_across_devices():
    """ncclAllGather across real devices (lamm_hip_comm_init_all over every visible GPU): each
    device computes its slab; every device's gathered C must be bit-identical (runs only where
    several GPUs are visible -- the driver's multi-GPU node)."""
    n = torch.cuda.device_count()
    devices = list(range(n))
    comm = la.Comm.all(devices)
    streams = []
    for d in devices:
        with torch.cuda.device(d):
            streams.append(torch.cuda.Stream())
    Cs, ref = _slabs_and_gather(comm, devices, ol.Q4_0, 4096, 4, 1024, devices, streams, seed=13)
    for c in Cs:
        np.testing.assert_array_equal(c, Cs[0])
    assert np.abs(Cs[0] - ref).max() <= 1e-3 * np.abs(ref).max()
    comm.close()


PREFILL = [(4096, 4096), (11008, 4096), (4096, 11008)]   # Llama-7B q/k/v/o, gate/up, down


@pytest.mark.parametrize("N", [16, 512])
@pytest.mark.parametrize("MK", PREFILL, ids=[f"{m}x{k}" for m, k in PREFILL])
def test_sharded_prefill_slabs_match_whole(MK, N):
    """Config 5's sharded prefill, node by node: every rank's slab GEMM
    (stationary weights, rows [r0, r0 + rows) of lamm_hip_shard_rows at llama-matmul-bench's
    16-row granularity, 2 and 8 ranks) against the same rows of the one-GPU call, from identical
    inputs, at the north-star tolerance |c - c_whole| <= 1e-3 sum |a b| per element.  A slab may
    run another tile plan (another fp32 summation order of the exact block dots) than the whole
    weight, so this is a tolerance, not bits; the whole call is pinned to the oracle on sampled
    rows."""
    M, K = MK
    t = ol.Q4_0
    A_q, B_q = _case(t, M, N, K, seed=M + N + K)
    arow = ORACLE.row_bytes(t, K)
    assert arow % 16 == 0
    A = torch.from_numpy(np.concatenate([A_q, np.zeros(64, np.uint8)])).cuda()
    B = torch.from_numpy(B_q.copy()).cuda()
    W = la.Weights(t, A, M, K)
    C = torch.full((N * M,), float("nan"), dtype=torch.float32, device="cuda")
    W.matmul_torch(B, C, N)
    torch.cuda.synchronize()
    whole = C.cpu().numpy().reshape(N, M)
    W.close()
    Ad = ORACLE.dequantize(t, A_q, M, K).astype(np.float64)
    Bd = ORACLE.dequantize(la.vec_dot_type(t), B_q, N, K).astype(np.float64)
    absdot = np.abs(Bd) @ np.abs(Ad).T
    rows_s = [0, 1, M // 2, M - 1]
    ref = ORACLE.mul_mat(t, len(rows_s), N, K, A_q.reshape(M, arow)[rows_s].reshape(-1), B_q)
    assert rel_err(whole[:, rows_s], ref, absdot[:, rows_s]).max() < TOL
    worst = 0.0
    for world in (2, 8):
        for r in range(world):
            r0, rows = la.shard_rows(M, world, r, 16)
            Ws = la.Weights(t, A[r0 * arow:], rows, K)
            slab = torch.full((rows * N,), float("nan"), dtype=torch.float32, device="cuda")
            Ws.matmul_torch(B, slab, N)
            torch.cuda.synchronize()
            got = slab.cpu().numpy().reshape(N, rows)
            Ws.close()
            err = rel_err(got, whole[:, r0:r0 + rows], absdot[:, r0:r0 + rows]).max()
            assert err < TOL, f"world {world} rank {r}: {err}"
            worst = max(worst, float(err))
    print(f"sharded prefill q4_0 {M}x{N}x{K}: worst slab vs whole {worst:.2e} of sum |a b|")
