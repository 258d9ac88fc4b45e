"""The reference's x86 float order on the GPU (csrc/lamm_ref.hip, lamm_hip_matmul_ex with
LAMM_ORDER_REFERENCE; q2_K / q4_K / q5_K since round 6): BIT-EXACT against the reference's own
lamm opt-3 AVX2 output (golden
C_lamm3, tools/gen_golden.py) and against the oracle's restatement of that order
(lo_mul_mat_avx, itself pinned to C_lamm3 in tests/test_oracle_golden.py), on ragged shapes,
strided operands and batch slices; and through the ggml boundary under LAMM_HIP_ORDER=reference."""
import os

import numpy as np
import pytest

from conftest import fixture_paths, load_fixture
import oracle_lib as ol

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
import lamm_amd as la  # noqa: E402
from test_gpu_parity import dev_bytes, pitch_blocks, pitched_A  # noqa: E402

ORACLE = ol.Oracle()
REF_TYPES = [ol.Q4_0, ol.Q4_1, ol.Q5_0, ol.Q5_1, ol.Q2_K, ol.Q4_K, ol.Q5_K, ol.Q6_K]


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


GOLD = [p for p in fixture_paths()
        if p.rsplit("/", 1)[-1].rsplit("_", 1)[0] in ("q4_0", "q4_1", "q5_0", "q5_1", "q2_k", "q4_k", "q5_k", "q6_k")]


@pytest.mark.parametrize("path", GOLD, ids=[p.rsplit("/", 1)[-1][:-4] for p in GOLD])
def test_reference_order_matches_lamm3_golden(path):
    """The golden blocks (A_q, the AVX2-quantized B) -> C bit for bit the reference's own lamm3
    output, on every row the reference computed (SURVEY §8a defect 1 leaves M % 4 rows unwritten)."""
    z = load_fixture(path)
    t, M, N, K = int(z["type"]), int(z["M"]), int(z["N"]), int(z["K"])
    c = ref_mul_mat(t, z["A_q"], z["B_avx"], M, N, K)[:N * M].reshape(N, M)
    done = M if t in (ol.Q4_K, ol.Q5_K, ol.Q6_K) else 4 * (M // 4)   # ggml's own loop: every row
    assert np.array_equal(bits(c[:, :done]), bits(z["C_lamm3"][:, :done]))


# N = 1: ref_gemv_kernel (chunks of 128 blocks: K = 11008 is 3; past 576 blocks ref_kernel)
SHAPES = [(1, 1, 256), (17, 3, 512), (31, 9, 768), (67, 1, 4096), (33, 18, 4096), (40, 7, 4096 + 256),
          (130, 2, 11008 - 256 * 3), (257, 33, 1024), (4096, 1, 4096), (45, 1, 11008), (13, 1, 4096 + 32 * 5),
          (40, 1, 32 * 600)]


def random_blocks(t, M, N, K, seed):
    rng = np.random.default_rng(seed)
    vt = la.vec_dot_type(t)
    if t in (ol.Q4_K, ol.Q5_K, ol.Q6_K):
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


@pytest.mark.parametrize("t", [ol.Q4_0, ol.Q2_K, ol.Q4_K, ol.Q5_K, ol.Q6_K], ids=["q4_0", "q2_k", "q4_k", "q5_k", "q6_k"])
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


GEMV_TYPES = [ol.Q4_0, ol.Q4_1, ol.Q5_0, ol.Q5_1]


@pytest.mark.parametrize("bpt", ["2", "4"])   # LAMM_REF_GEMV_BPT: blocks per producer thread
@pytest.mark.parametrize("t", GEMV_TYPES, ids=[ol.NAMES[t] for t in GEMV_TYPES])
@pytest.mark.parametrize("shape", [(1, 256), (67, 4096), (4096, 4096), (45, 11008), (9, 32 * 577), (13, 4096 + 32 * 5)],
                         ids=["1x256", "67x4096", "4096x4096", "45x11008", "9x18464", "13x4256"])
def test_reference_order_gemv_f32_rows(t, shape, bpt, monkeypatch):
    """One F32 activation row (the boundary's decode calls, kFused): ref_gemv_kernel quantizes it
    in its staging the way ggml's AVX2 INIT does, then computes in the reference's order -- the
    same bits as quantizing with the oracle's AVX2 flavour and running mul_mat_avx.  Past 576
    blocks the kernel declines F32 rows (LammError), as the boundary's routing expects.  Both
    producer widths (2 or 4 blocks per thread: 512 / 256 threads per workgroup); 13x4256: an odd
    block count (a partial last producer span)."""
    monkeypatch.setenv("LAMM_REF_GEMV_BPT", bpt)
    M, K = shape
    rng = np.random.default_rng(M + K)
    A_q = ORACLE.quantize(t, rng.standard_normal((M, K), dtype=np.float32), ol.QUANT_REF)
    x = (rng.standard_normal((1, K)) * rng.uniform(0.1, 3.0)).astype(np.float32)
    x[0, :7] = 0.0                       # a zero run inside the first block
    kb = K // 32
    lda = pitch_blocks(t, kb)
    A = dev_bytes(pitched_A(t, A_q, M, kb, lda))
    B = torch.from_numpy(x.reshape(-1)).to("cuda")
    C = torch.full((M + 16,), float("nan"), dtype=torch.float32, device="cuda")
    Am = la.Matrix(A.data_ptr(), t, M, kb, lda)
    Bm = la.Matrix(B.data_ptr(), la.F32, K, 1, K)
    Cm = la.Matrix(C.data_ptr(), la.F32, M, 1, M)
    if kb > 576:
        with pytest.raises(la.LammError):
            la.matmul_ex(Am, Bm, Cm, None, la.ORDER_REFERENCE, torch.cuda.current_stream().cuda_stream)
        return
    la.matmul_ex(Am, Bm, Cm, None, la.ORDER_REFERENCE, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    got = C.cpu().numpy()[:M]
    B_q = ORACLE.quantize(la.vec_dot_type(t), x, ol.QUANT_AVX)
    want = ORACLE.mul_mat_avx(t, M, 1, K, A_q, B_q)[0]
    assert np.array_equal(bits(got), bits(want)), f"{(got != want).sum()} of {M} differ"


@pytest.mark.parametrize("t", [ol.Q4_0, ol.Q5_1], ids=["q4_0", "q5_1"])
def test_reference_order_gemv_slices(t):
    """N = 1 over 3 x 2 batch slices (one A slice per 3 B slices): ref_gemv_kernel's slice path."""
    M, N, K = 37, 1, 4096
    kb = K // 32
    lda = pitch_blocks(t, kb)
    vt = la.vec_dot_type(t)
    rbB = kb * la.type_size(vt)
    A_q = [random_blocks(t, M, 1, K, seed=20 + s)[0] for s in range(2)]
    B_q = [random_blocks(t, 1, N, K, seed=30 + s)[1] for s in range(6)]
    arow = lda * la.type_size(t)
    bt = la.Batch(2, 1, 6, 1, M * arow, 2 * M * arow, N * rbB, 6 * N * rbB, 4 * M * N, 4 * M * N * 6)
    A = dev_bytes(np.concatenate([pitched_A(t, A_q[s], M, kb, lda)[:M * arow] for s in range(2)] +
                                 [np.zeros(64, np.uint8)]))
    B = dev_bytes(np.concatenate(B_q))
    C = torch.full((6 * M + 16,), float("nan"), dtype=torch.float32, device="cuda")
    la.mul_mat_torch(t, A, B, C, M, N, K, lda=lda, batch=bt, flags=la.ORDER_REFERENCE)
    torch.cuda.synchronize()
    got = C.cpu().numpy()
    for z in range(6):
        want = ORACLE.mul_mat_avx(t, M, N, K, A_q[z // 3], B_q[z])[0]
        assert np.array_equal(bits(got[z * M:(z + 1) * M]), bits(want)), f"slice {z}"


F16_NODES = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ref_nodes", "f16_attention.npz")


@pytest.mark.parametrize("tag", ["prefill_kq", "prefill_kqv", "decode_kq", "decode_kqv"])
def test_reference_order_f16_matches_reference_attention_nodes(tag):
    """F16 x F16 (ref_f16_kernel, ggml_vec_dot_f16's AVX2 order): the reference's own KQ / KQV
    nodes (tools/gen_golden_f16.py: its CPU build, 4 heads) bit for bit, the heads as batch slices."""
    z = np.load(F16_NODES, allow_pickle=False)
    A16, X, Cref = z[tag + "_src0"], z[tag + "_src1"], z[tag + "_dst"]
    heads, M, K = A16.shape
    N = X.shape[1]
    B = np.concatenate([ORACLE.quantize(ol.F16, X[h], ol.QUANT_REF) for h in range(heads)])
    A = dev_bytes(np.concatenate([A16.reshape(-1).view(np.uint8), np.zeros(64, np.uint8)]))
    Bd = dev_bytes(np.concatenate([B, np.zeros(64, np.uint8)]))
    C = torch.full((heads * N * M + 16,), float("nan"), dtype=torch.float32, device="cuda")
    bt = la.Batch(heads, 1, heads, 1, 2 * M * K, 2 * M * K * heads, 2 * N * K, 2 * N * K * heads, 4 * M * N,
                  4 * M * N * heads)
    la.mul_mat_torch(la.F16, A, Bd, C, M, N, K, batch=bt, flags=la.ORDER_REFERENCE)
    torch.cuda.synchronize()
    got = C.cpu().numpy()[:heads * N * M].reshape(heads, N, M)
    assert np.array_equal(bits(got), bits(np.ascontiguousarray(Cref))), f"{(got != Cref).sum()} differ"


@pytest.mark.parametrize("shape", [(64, 40, 128), (33, 7, 100), (128, 1, 64), (97, 65, 544), (5, 3, 20), (32, 32, 4096)],
                         ids=["64x40x128", "33x7x100", "128x1x64", "97x65x544", "5x3x20", "32x32x4096"])
def test_reference_order_f16_vs_oracle(shape):
    """Ragged tiles, n % 32 leftovers (added in double after the tree), the 2-byte-load staging
    (K = 100, 20: rows not 16-byte multiples) and f16 subnormals in both operands."""
    M, N, K = shape
    rng = np.random.default_rng(M * 3 + N * 5 + K)
    a = (rng.standard_normal((M, K)) * 0.5).astype(np.float16)
    b32 = (rng.standard_normal((N, K)) * 2.0).astype(np.float32)
    a.reshape(-1)[::17] = np.float16(3e-6)            # f16 subnormals
    b32.reshape(-1)[::13] = 1e-7
    lda = (K + 7) // 8 * 8
    ap = np.zeros((M, lda), np.float16)
    ap[:, :K] = a
    B = ORACLE.quantize(ol.F16, b32, ol.QUANT_REF)
    A = dev_bytes(np.concatenate([ap.reshape(-1).view(np.uint8), np.zeros(64, np.uint8)]))
    Bd = dev_bytes(np.concatenate([B, np.zeros(64, np.uint8)]))
    C = torch.full((N * M + 16,), float("nan"), dtype=torch.float32, device="cuda")
    la.mul_mat_torch(la.F16, A, Bd, C, M, N, K, lda=lda, flags=la.ORDER_REFERENCE)
    torch.cuda.synchronize()
    got = C.cpu().numpy()[:N * M].reshape(N, M)
    want = ORACLE.mul_mat_avx(ol.F16, M, N, K, a.view(np.uint8).reshape(M, 2 * K), B)
    assert np.array_equal(bits(got), bits(want)), f"{(got != want).sum()} of {got.size} differ"


def test_reference_order_rejects_other_types():
    """q8_0: lamm's AVX2 q8_0 kernel is SURVEY §8a defect 2 (signed weights through maddubs), an
    order not worth reproducing -- the reference-order flag refuses it (the boundary then keeps the
    fast engines for it)."""
    M, N, K = 16, 2, 256
    for t, vt in ((ol.Q8_0, ol.Q8_0),):
        A = torch.zeros(M * la.row_bytes(t, K) + 64, dtype=torch.uint8, device="cuda")
        B = torch.zeros(N * la.row_bytes(vt, K) + 64, dtype=torch.uint8, device="cuda")
        C = torch.zeros(N * M, dtype=torch.float32, device="cuda")
        with pytest.raises(la.LammError):
            la.mul_mat_torch(t, A, B, C, M, N, K, flags=la.ORDER_REFERENCE)


PREFILL_KERNELS = ["1", "2", "3", "4", "5", "6"]   # LAMM_REF_MFMA: ref_mfma / ref_mfma2 G=2 / G=1 / G=4 / G=2 swizzled / + interleaved


@pytest.mark.parametrize("variant", PREFILL_KERNELS)
@pytest.mark.parametrize("t", [ol.Q4_0, ol.Q4_1, ol.Q5_0, ol.Q5_1], ids=["q4_0", "q4_1", "q5_0", "q5_1"])
@pytest.mark.parametrize("shape", [(70, 40, 512), (128, 96, 1056), (64, 9, 256)], ids=["70x40x512", "128x96x1056", "64x9x256"])
def test_reference_order_prefill_kernels_bit_exact(variant, t, shape, monkeypatch):
    """Every reference-order prefill kernel (lamm_ref.hip; LAMM_REF_MFMA selects it) computes the
    reference's lane order bit for bit: ragged row / column tiles, K not a multiple of the 8-block
    chunk, and the swizzled activation image (=5)."""
    monkeypatch.setenv("LAMM_REF_MFMA", variant)
    M, N, K = shape
    A_q, B_q = random_blocks(t, M, N, K, seed=M * 3 + N * 17 + K + int(variant))
    c = ref_mul_mat(t, A_q, B_q, M, N, K)[:N * M].reshape(N, M)
    want = ORACLE.mul_mat_avx(t, M, N, K, A_q, B_q)
    assert np.array_equal(bits(c), bits(want)), f"{(c != want).sum()} of {c.size} differ"


KQ_REF = [ol.Q2_K, ol.Q4_K, ol.Q5_K]


@pytest.mark.parametrize("t", KQ_REF, ids=[ol.NAMES[t] for t in KQ_REF])
@pytest.mark.parametrize("shape", [(300, 64, 1024), (4096, 32, 4096)], ids=["300x64x1024", "4096x32x4096"])
def test_reference_order_kquants_prefill_bit_exact(t, shape):
    """q2_K (lamm's AVX2 block kernel) / q4_K / q5_K (ggml's AVX2 vec_dot) at prefill-sized N through
    ref_kernel's 8-column tiles: sampled rows bit for bit against the oracle's restatement."""
    M, N, K = shape
    A_q, B_q = random_blocks(t, M, N, K, seed=M + N + K + t)
    c = ref_mul_mat(t, A_q, B_q, M, N, K)[:N * M].reshape(N, M)
    rows = np.unique(np.r_[np.random.default_rng(M).choice(M, 64, replace=False), [0, M - 1]])
    arow = la.row_bytes(t, K)
    A_s = np.concatenate([A_q[r * arow:(r + 1) * arow] for r in rows])
    want = ORACLE.mul_mat_avx(t, len(rows), N, K, A_s, B_q)
    got = c[:, rows]
    assert np.array_equal(bits(got), bits(want)), f"{(got != want).sum()} of {got.size} differ"


FULL_SHAPES = [(4096, 512, 4096), (11008, 512, 4096)]


@pytest.mark.parametrize("t", [ol.Q4_0, ol.Q4_1, ol.Q5_0, ol.Q5_1], ids=["q4_0", "q4_1", "q5_0", "q5_1"])
@pytest.mark.parametrize("shape", FULL_SHAPES, ids=[f"{m}x{n}x{k}" for m, n, k in FULL_SHAPES])
def test_reference_order_prefill_full_size(t, shape):
    """The reference-order prefill kernel the boundary runs for a pp512 call (the swizzled ref_mfma2
    for q4_0 / q4_1 / q5_0, ref_mfma for q5_1) at config 3's shape and at Llama-7B's ffn shape:
    256 sampled weight rows x all 512 columns, bit for bit against the oracle's restatement of the
    reference's AVX2 lane order."""
    if t != ol.Q4_0 and shape[0] != 4096:
        pytest.skip("the ffn shape runs for q4_0, Llama-7B's projection format")
    M, N, K = shape
    A_q, B_q = random_blocks(t, M, N, K, seed=M + N + K + t)
    c = ref_mul_mat(t, A_q, B_q, M, N, K)[:N * M].reshape(N, M)
    rows = np.sort(np.random.default_rng(M).choice(M, 256, replace=False))
    arow = la.row_bytes(t, K)
    A_s = np.concatenate([A_q[r * arow:(r + 1) * arow] for r in rows])
    want = ORACLE.mul_mat_avx(t, len(rows), N, K, A_s, B_q)
    got = c[:, rows]
    assert np.array_equal(bits(got), bits(want)), f"{(got != want).sum()} of {got.size} differ"
