"""The reference's x86 float order on the GPU (csrc/lamm_ref.hip, lamm_hip_matmul_ex with
LAMM_ORDER_REFERENCE): BIT-EXACT against the reference's own lamm opt-3 AVX2 output (golden
C_lamm3, tools/gen_golden.py) and against the oracle's restatement of that order
(lo_mul_mat_avx, itself pinned to C_lamm3 in tests/test_oracle_golden.py), on ragged shapes,
strided operands and batch slices; and through the ggml boundary, which runs this order by
default (LAMM_HIP_ORDER)."""
import numpy as np
import pytest

from conftest import fixture_paths, load_fixture
import oracle_lib as ol

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
import lamm_amd as la  # noqa: E402
from test_gpu_parity import dev_bytes, pitch_blocks, pitched_A  # noqa: E402

ORACLE = ol.Oracle()
REF_TYPES = [ol.Q4_0, ol.Q4_1, ol.Q5_0, ol.Q5_1, ol.Q6_K]


def ref_mul_mat(t, A_q, B_q, M, N, K):
    kb = K // la.blck_size(t)
    lda = pitch_blocks(t, kb)
    A = dev_bytes(pitched_A(t, A_q, M, kb, lda))
    B = dev_bytes(B_q)
    C = torch.full((N * M + 16,), float("nan"), dtype=torch.float32, device="cuda")
    la.mul_mat_torch(t, A, B, C, M, N, K, lda=lda, flags=la.ORDER_REFERENCE)
    torch.cuda.synchronize()
    return C.cpu().numpy()


def bits(x):
    return np.ascontiguousarray(x, dtype=np.float32).view(np.uint32)


GOLD = [p for p in fixture_paths() if p.rsplit("/", 1)[-1].rsplit("_", 1)[0] in ("q4_0", "q4_1", "q5_0", "q5_1", "q6_k")]


@pytest.mark.parametrize("path", GOLD, ids=[p.rsplit("/", 1)[-1][:-4] for p in GOLD])
def test_reference_order_matches_lamm3_golden(path):
    """The golden blocks (A_q, the AVX2-quantized B) -> C bit for bit the reference's own lamm3
    output, on every row the reference computed (SURVEY §8a defect 1 leaves M % 4 rows unwritten)."""
    z = load_fixture(path)
    t, M, N, K = int(z["type"]), int(z["M"]), int(z["N"]), int(z["K"])
    c = ref_mul_mat(t, z["A_q"], z["B_avx"], M, N, K)[:N * M].reshape(N, M)
    done = M if t == ol.Q6_K else 4 * (M // 4)
    assert np.array_equal(bits(c[:, :done]), bits(z["C_lamm3"][:, :done]))


SHAPES = [(1, 1, 256), (17, 3, 512), (31, 9, 768), (67, 1, 4096), (33, 18, 4096), (40, 7, 4096 + 256),
          (130, 2, 11008 - 256 * 3), (257, 33, 1024), (4096, 1, 4096)]


def random_blocks(t, M, N, K, seed):
    rng = np.random.default_rng(seed)
    vt = la.vec_dot_type(t)
    if t == ol.Q6_K:
        A_q = ol.random_kq_blocks(t, M, K, rng)
    else:
        A_q = ORACLE.quantize(t, rng.standard_normal((M, K), dtype=np.float32), ol.QUANT_REF)
    B_q = ORACLE.quantize(vt, rng.standard_normal((N, K), dtype=np.float32),
                          ol.QUANT_AVX if vt in (ol.Q8_0, ol.Q8_1) else ol.QUANT_REF)
    return A_q, B_q


@pytest.mark.parametrize("t", REF_TYPES, ids=[ol.NAMES[t] for t in REF_TYPES])
@pytest.mark.parametrize("shape", SHAPES, ids=[f"{m}x{n}x{k}" for m, n, k in SHAPES])
def test_reference_order_vs_oracle_bit_exact(t, shape):
    M, N, K = shape
    if K % la.blck_size(t):
        pytest.skip("K not a multiple of the super-block")
    A_q, B_q = random_blocks(t, M, N, K, seed=M * 7 + N * 131 + K)
    c = ref_mul_mat(t, A_q, B_q, M, N, K)[:N * M].reshape(N, M)
    want = ORACLE.mul_mat_avx(t, M, N, K, A_q, B_q)
    assert np.array_equal(bits(c), bits(want)), f"{(c != want).sum()} of {c.size} differ"


@pytest.mark.parametrize("t", [ol.Q4_0, ol.Q6_K], ids=["q4_0", "q6_k"])
def test_reference_order_strides_and_slices(t):
    """Pitched A rows, ldc > M, and 3 x 2 batch slices broadcasting one A slice over 3 B slices
    (ggml's r2 = ne12 / ne02): every slice bit-exact."""
    M, N, K = 45, 10, 512
    kb = K // la.blck_size(t)
    lda = pitch_blocks(t, kb + 1)   # a pitch past the row, still 16-byte aligned
    vt = la.vec_dot_type(t)
    rbB = kb * la.type_size(vt)
    A_q = [random_blocks(t, M, 1, K, seed=s)[0] for s in range(2)]   # ne02 = 2 A slices
    B_q = [random_blocks(t, 1, N, K, seed=10 + s)[1] for s in range(6)]
    arow = lda * la.type_size(t)
    ldc = M + 3
    bt = la.Batch(2, 1, 6, 1, M * arow, 2 * M * arow, N * rbB, 6 * N * rbB, 4 * ldc * N, 4 * ldc * N * 6)
    A = dev_bytes(np.concatenate([pitched_A(t, A_q[s], M, kb, lda)[:M * arow] for s in range(2)] +
                                 [np.zeros(64, np.uint8)]))
    B = dev_bytes(np.concatenate(B_q))
    C = torch.full((6 * N * ldc + 16,), float("nan"), dtype=torch.float32, device="cuda")
    la.mul_mat_torch(t, A, B, C, M, N, K, lda=lda, ldc=ldc, batch=bt, flags=la.ORDER_REFERENCE)
    torch.cuda.synchronize()
    got = C.cpu().numpy()
    for z in range(6):
        want = ORACLE.mul_mat_avx(t, M, N, K, A_q[z // 3], B_q[z])
        sl = got[z * N * ldc:(z + 1) * N * ldc].reshape(N, ldc)[:, :M]
        assert np.array_equal(bits(sl), bits(want)), f"slice {z}"


def test_reference_order_rejects_other_types():
    M, N, K = 16, 2, 256
    for t, vt in ((ol.Q8_0, ol.Q8_0), (ol.Q2_K, ol.Q8_K), (ol.Q4_K, ol.Q8_K)):
        A = torch.zeros(M * la.row_bytes(t, K) + 64, dtype=torch.uint8, device="cuda")
        B = torch.zeros(N * la.row_bytes(vt, K) + 64, dtype=torch.uint8, device="cuda")
        C = torch.zeros(N * M, dtype=torch.float32, device="cuda")
        with pytest.raises(la.LammError):
            la.mul_mat_torch(t, A, B, C, M, N, K, flags=la.ORDER_REFERENCE)
