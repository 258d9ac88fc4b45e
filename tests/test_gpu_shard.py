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
