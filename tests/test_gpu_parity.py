"""GPU parity: the HIP path (called through the C ABI) vs the pinned oracle and the
reference's own golden vectors.

Tolerance (BASELINE.json north star): per output
    |c_gpu - c_ref| <= 1e-3 * max(|c_ref|, sum_k |a_k b_k|)
Per-block int32 dots are exact on both sides; only the fp32 accumulation order of
the d_a*d_b*S terms differs, so observed errors are ~1e-7.
"""
import numpy as np
import pytest

from conftest import fixture_paths, load_fixture, load_inputs, rel_err
import oracle_lib as ol

pytestmark = pytest.mark.gpu
TOL = 1e-3

torch = pytest.importorskip("torch")
import lamm_amd as la  # noqa: E402

ORACLE = ol.Oracle()
FIXTURES = fixture_paths()


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available() or la.device_count() == 0:
        pytest.fail("GPU tests need a gfx950 device (run with -m 'not gpu' on CPU)")
    yield


def pitch_blocks(t, kb):
    """smallest lda (blocks) >= kb whose byte pitch is a multiple of 16"""
    bpb = la.type_size(t)
    lda = kb
    while (lda * bpb) % 16:
        lda += 1
    return lda


def dev_bytes(arr):
    return torch.from_numpy(np.ascontiguousarray(arr).view(np.uint8).reshape(-1).copy()).cuda()


def pitched_A(t, A_q, M, kb, lda):
    rb = kb * la.type_size(t)
    out = np.zeros(M * lda * la.type_size(t) + 64, np.uint8)
    src = np.ascontiguousarray(A_q).reshape(M, rb)
    out[:M * lda * la.type_size(t)].reshape(M, lda * la.type_size(t))[:, :rb] = src
    return out


def gpu_mul_mat(t, A_q, B_q, M, N, K, ldc=None, lda=None, ldb=None):
    kb = K // la.blck_size(t)
    vt = la.vec_dot_type(t)
    lda = lda or pitch_blocks(t, kb)
    A = dev_bytes(pitched_A(t, A_q, M, kb, lda))
    if ldb is not None and ldb != kb:
        rb = kb * la.type_size(vt)
        Bp = np.zeros(N * ldb * la.type_size(vt), np.uint8)
        Bp.reshape(N, -1)[:, :rb] = np.ascontiguousarray(B_q).reshape(N, rb)
        B = dev_bytes(Bp)
    else:
        B = dev_bytes(B_q)
    ldc = ldc or M
    C = torch.full((N * ldc + 16,), float("nan"), dtype=torch.float32, device="cuda")
    la.mul_mat_torch(t, A, B, C, M, N, K, lda=lda, ldb=ldb, ldc=ldc)
    torch.cuda.synchronize()
    c = C.cpu().numpy()
    return np.stack([c[j * ldc:j * ldc + M] for j in range(N)]), c


def absdot(t, A_q, B_q, M, N, K):
    Ad = ORACLE.dequantize(t, A_q, M, K).astype(np.float64)
    Bd = ORACLE.dequantize(la.vec_dot_type(t), B_q, N, K).astype(np.float64)
    return np.abs(Bd) @ np.abs(Ad).T


def _ids(paths):
    return [p.rsplit("/", 1)[-1][:-4] for p in paths]


@pytest.mark.parametrize("path", FIXTURES, ids=_ids(FIXTURES))
def test_golden_vectors(path):
    """Same bytes as the reference: C_scalar (from_float_reference B) and the
    stock AVX2 vec_dot output (AVX2 from_float B)."""
    z = load_fixture(path)
    t, M, N, K = int(z["type"]), int(z["M"]), int(z["N"]), int(z["K"])
    c_ref, _ = gpu_mul_mat(t, z["A_q"], z["B_ref"], M, N, K)
    assert np.isfinite(c_ref).all()
    e1 = rel_err(c_ref, z["C_scalar"], z["absdot"]).max()
    c_avx, _ = gpu_mul_mat(t, z["A_q"], z["B_avx"], M, N, K)
    e2 = rel_err(c_avx, z["C_vdot_avx"], z["absdot"]).max()
    print(f"{z['name']}: max rel err vs scalar {e1:.2e}, vs avx2 {e2:.2e}")
    assert e1 < TOL and e2 < TOL


def random_case(t, M, N, K, seed, flavour=ol.QUANT_AVX):
    rng = np.random.default_rng(seed)
    a = rng.standard_normal((M, K), dtype=np.float32)
    b = rng.standard_normal((N, K), dtype=np.float32)
    vt = la.vec_dot_type(t)
    A_q = ORACLE.quantize(t, a, ol.QUANT_REF)
    fl = flavour if vt in (ol.Q8_0, ol.Q8_1) else ol.QUANT_REF
    B_q = ORACLE.quantize(vt, b, fl)
    return A_q, B_q


SHAPES = [(1, 1, 256), (17, 3, 512), (31, 5, 768), (16, 8, 4096), (40, 7, 4096 + 256), (5, 9, 256),
          (33, 17, 1024), (130, 2, 8192 + 512)]


@pytest.mark.parametrize("t", ol.A_TYPES, ids=[ol.NAMES[t] for t in ol.A_TYPES])
@pytest.mark.parametrize("shape", SHAPES, ids=[f"{m}x{n}x{k}" for m, n, k in SHAPES])
def test_random_shapes_vs_oracle(t, shape):
    """Ragged M (not a multiple of the 16-row tile), N across the GEMV (<=8) and
    grouped/GEMM (>8) paths, K spanning several 4096-element segments."""
    M, N, K = shape
    A_q, B_q = random_case(t, M, N, K, seed=M * 1000 + N * 10 + K)
    c, _ = gpu_mul_mat(t, A_q, B_q, M, N, K)
    ref = ORACLE.mul_mat(t, M, N, K, A_q, B_q)
    err = rel_err(c, ref, absdot(t, A_q, B_q, M, N, K)).max()
    assert err < TOL, err


KQ_SHAPES = [(1, 1, 256), (17, 3, 512), (40, 7, 4096 + 256), (33, 17, 1024), (130, 2, 8192 + 512), (4096, 1, 4096)]


@pytest.mark.parametrize("t", ol.KQ_TYPES, ids=[ol.NAMES[t] for t in ol.KQ_TYPES])
@pytest.mark.parametrize("shape", KQ_SHAPES, ids=[f"{m}x{n}x{k}" for m, n, k in KQ_SHAPES])
def test_kquants_random_bytes_vs_oracle(t, shape):
    """SURVEY §8f q4_K / q5_K / q6_K (beyond the reference's lamm set): random block bytes
    (finite fp16 scales) against q8_K rows from the oracle's quantizer; GEMV (N <= 8), the
    grouped-GEMV path (N > 8), K spanning several 4096-element segments."""
    M, N, K = shape
    rng = np.random.default_rng(M * 31 + N * 7 + K + t)
    A_q = ol.random_kq_blocks(t, M, K, rng)
    B_q = ORACLE.quantize(ol.Q8_K, rng.standard_normal((N, K), dtype=np.float32))
    c, _ = gpu_mul_mat(t, A_q, B_q, M, N, K)
    ref = ORACLE.mul_mat(t, M, N, K, A_q, B_q)
    err = rel_err(c, ref, absdot(t, A_q, B_q, M, N, K)).max()
    assert err < TOL, err


KQG_SHAPES = [(130, 129, 2048), (64, 300, 256), (257, 40, 1024), (9, 9, 512)]
KQG_TYPES = ol.KQ_TYPES + [ol.Q2_K]   # q2_K shares the super-block GEMM engine


@pytest.mark.parametrize("t", KQG_TYPES, ids=[ol.NAMES[t] for t in KQG_TYPES])
@pytest.mark.parametrize("shape", KQG_SHAPES, ids=[f"{m}x{n}x{k}" for m, n, k in KQG_SHAPES])
def test_kquant_gemm_vs_oracle(t, shape, monkeypatch):
    """The k-quant prefill GEMM (lamm_gemm_kq.hip: integer sub-block scales folded into the
    weight operand, split exactly into two int8 planes): ragged M / N against its 64 x 128
    tile, several super-blocks, row pitch padding; the grouped GEMV (LAMM_KQ_GEMM=0) must
    agree within the same tolerance."""
    M, N, K = shape
    rng = np.random.default_rng(M * 13 + N * 5 + K + t)
    A_q = ol.random_kq_blocks(t, M, K, rng)
    B_q = ORACLE.quantize(ol.Q8_K, rng.standard_normal((N, K), dtype=np.float32))
    ref = ORACLE.mul_mat(t, M, N, K, A_q, B_q)
    den = absdot(t, A_q, B_q, M, N, K)
    kb = K // 256
    c, raw = gpu_mul_mat(t, A_q, B_q, M, N, K, lda=pitch_blocks(t, kb + 1), ldc=M + 5)
    assert rel_err(c, ref, den).max() < TOL
    assert np.isnan(np.concatenate([raw[j * (M + 5) + M:(j + 1) * (M + 5)] for j in range(N)])).all()
    monkeypatch.setenv("LAMM_KQ_GEMM", "0")
    c2, _ = gpu_mul_mat(t, A_q, B_q, M, N, K)
    assert rel_err(c2, ref, den).max() < TOL


@pytest.mark.parametrize("variant", ["0", "1"], ids=["dma", "simple"])
@pytest.mark.parametrize("t", KQG_TYPES, ids=[ol.NAMES[t] for t in KQG_TYPES])
def test_kquant_gemm_variants_and_stationary(t, variant, monkeypatch):
    """Both k-quant GEMM kernels (LAMM_KQ_VARIANT) and the weight-stationary handle (packed
    planes made once) against the oracle; the handle's bytes equal the per-call path's."""
    monkeypatch.setenv("LAMM_KQ_VARIANT", variant)
    M, N, K = 200, 150, 1536
    rng = np.random.default_rng(t * 3 + int(variant))
    A_q = ol.random_kq_blocks(t, M, K, rng)
    B_q = ORACLE.quantize(ol.Q8_K, rng.standard_normal((N, K), dtype=np.float32))
    ref = ORACLE.mul_mat(t, M, N, K, A_q, B_q)
    c, _ = gpu_mul_mat(t, A_q, B_q, M, N, K)
    assert rel_err(c, ref, absdot(t, A_q, B_q, M, N, K)).max() < TOL
    kb = K // 256
    lda = pitch_blocks(t, kb)
    A = dev_bytes(np.concatenate([pitched_A(t, A_q, M, kb, lda), np.zeros(64, np.uint8)]))
    B = dev_bytes(B_q)
    W = la.Weights(t, A, M, K, lda=lda)
    assert W.packed_bytes > 0
    C0 = torch.full((N * M,), float("nan"), dtype=torch.float32, device="cuda")
    C1 = torch.full_like(C0, float("nan"))
    la.mul_mat_torch(t, A, B, C0, M, N, K, lda=lda)
    W.matmul_torch(B, C1, N)
    torch.cuda.synchronize()
    assert torch.equal(C0, C1)
    W.close()


@pytest.mark.parametrize("t", KQG_TYPES, ids=[ol.NAMES[t] for t in KQG_TYPES])
def test_kquant_gemm_extremes_and_broadcast(t):
    """Extreme operands: every weight byte 0xFF / 0x00 patterns with the largest scales
    (q6_K: sc = -128, q - 32 = -32 -> A' = 4096, the top of the hi/lo split) against q8_K
    quants of +-127, and a ggml broadcast (2 weight slices over 4 activation slices)."""
    M, N, K = 70, 33, 512
    bpb = {ol.Q4_K: 144, ol.Q5_K: 176, ol.Q6_K: 210, ol.Q2_K: 84}[t]
    rng = np.random.default_rng(t)
    As = []
    for s in range(2):
        blk = np.full((M * K // 256, bpb), 0xFF if s == 0 else 0x00, np.uint8)
        if t == ol.Q6_K:
            blk[:, 192:208] = 0x80                       # int8 scale -128
        for off in ol.FP16_FIELDS[t]:
            blk[:, off:off + 2] = np.array([0.01], np.float16).view(np.uint8)
        As.append(blk.reshape(-1))
    x = np.where(rng.random((4 * N, K)) < 0.5, -1.0, 1.0).astype(np.float32)
    Bs = [ORACLE.quantize(ol.Q8_K, x[s * N:(s + 1) * N]) for s in range(4)]
    kb = K // 256
    lda = pitch_blocks(t, kb)
    abytes = M * lda * bpb
    A = dev_bytes(np.concatenate([pitched_A(t, a, M, kb, lda)[:abytes] for a in As] + [np.zeros(64, np.uint8)]))
    bbytes = N * kb * 292
    B = dev_bytes(np.concatenate(Bs))
    C = torch.full((4 * N * M,), float("nan"), dtype=torch.float32, device="cuda")
    bt = la.Batch(2, 1, 4, 1, abytes, 2 * abytes, bbytes, 4 * bbytes, 4 * M * N, 4 * M * N * 4)
    la.mul_mat_torch(t, A, B, C, M, N, K, lda=lda, batch=bt)
    torch.cuda.synchronize()
    c = C.cpu().numpy().reshape(4, N, M)
    for z in range(4):
        a = As[z // 2]
        ref = ORACLE.mul_mat(t, M, N, K, a, Bs[z])
        assert rel_err(c[z], ref, absdot(t, a, Bs[z], M, N, K)).max() < TOL, z


FP6_TYPES = [ol.Q4_0, ol.Q4_1, ol.Q5_0]
GEMM_SHAPES = [(33, 17, 1024), (130, 9, 8192 + 512), (257, 129, 4096 + 64), (300, 40, 96)]


DQ_TYPES = [ol.Q4_0, ol.Q4_1, ol.Q5_0, ol.Q5_1, ol.Q8_0]
ENGINE_CASES = [(t, e) for e in ("fp6", "i8") for t in FP6_TYPES] + [(t, "dq16") for t in DQ_TYPES]


@pytest.mark.parametrize("t,engine", ENGINE_CASES, ids=[f"{ol.NAMES[t]}-{e}" for t, e in ENGINE_CASES])
@pytest.mark.parametrize("shape", GEMM_SHAPES, ids=[f"{m}x{n}x{k}" for m, n, k in GEMM_SHAPES])
def test_gemm_engines_vs_oracle(t, shape, engine, monkeypatch):
    """The prefill engines (LAMM_GEMM_PATH: block-scaled fp6 MFMA / MFMA-i8 / the dequantizing f16
    engine of every 32-element format) on ragged shapes: M and N not multiples of the 256x128 /
    128x64 tiles, K not a multiple of the K-step or of dq16's 4-block quads (odd block counts: K=96
    is 3 blocks, 4160 is 130)."""
    monkeypatch.setenv("LAMM_GEMM_PATH", engine)
    if engine == "dq16":
        assert la.gemm_engine(t, *shape) == "dq16"
    M, N, K = shape
    A_q, B_q = random_case(t, M, N, K, seed=M * 7 + N * 3 + K)
    c, _ = gpu_mul_mat(t, A_q, B_q, M, N, K)
    ref = ORACLE.mul_mat(t, M, N, K, A_q, B_q)
    err = rel_err(c, ref, absdot(t, A_q, B_q, M, N, K)).max()
    assert err < TOL, err


@pytest.mark.parametrize("t", DQ_TYPES, ids=[ol.NAMES[t] for t in DQ_TYPES])
def test_gemm_dq16_batched_strided(t, monkeypatch):
    """dq16 with ggml batch dims (2 weight slices broadcast over 4 activation slices, r2 = 2), a
    padded C pitch (untouched tail stays NaN) and padded A / B row pitches."""
    monkeypatch.setenv("LAMM_GEMM_PATH", "dq16")
    M, N, K, ne02, ne12 = 200, 70, 1024 + 160, 2, 4
    vt = la.vec_dot_type(t)
    kb = K // 32
    lda, ldb, ldc = pitch_blocks(t, kb + 1), kb + 3, M + 5   # A pitches stay 16-byte multiples
    arow, brow = lda * la.type_size(t), ldb * la.type_size(vt)
    rng = np.random.default_rng(5 + t)
    As = [ORACLE.quantize(t, rng.standard_normal((M, K), dtype=np.float32), ol.QUANT_REF) for _ in range(ne02)]
    Bs = [ORACLE.quantize(vt, rng.standard_normal((N, K), dtype=np.float32), ol.QUANT_AVX) for _ in range(ne12)]
    Ap = np.zeros((ne02, M, arow), np.uint8)
    for a in range(ne02):
        Ap[a, :, :kb * la.type_size(t)] = As[a].reshape(M, -1)
    Bp = np.zeros((ne12, N, brow), np.uint8)
    for z in range(ne12):
        Bp[z, :, :kb * la.type_size(vt)] = Bs[z].reshape(N, -1)
    A = dev_bytes(np.concatenate([Ap.reshape(-1), np.zeros(64, np.uint8)]))
    B = dev_bytes(Bp)
    C = torch.full((ne12 * N * ldc,), float("nan"), dtype=torch.float32, device="cuda")
    bt = la.Batch(ne02, 1, ne12, 1, M * arow, ne02 * M * arow, N * brow, ne12 * N * brow, 4 * N * ldc,
                  4 * ne12 * N * ldc)
    la.matmul_batched(la.Matrix(A.data_ptr(), t, M, kb, lda), la.Matrix(B.data_ptr(), vt, kb, N, ldb),
                      la.Matrix(C.data_ptr(), la.F32, M, N, ldc), bt, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    c = C.cpu().numpy().reshape(ne12, N, ldc)
    assert np.isnan(c[:, :, M:]).all()
    for z in range(ne12):
        a = As[z // (ne12 // ne02)]
        ref = ORACLE.mul_mat(t, M, N, K, a, Bs[z])
        assert rel_err(c[z, :, :M], ref, absdot(t, a, Bs[z], M, N, K)).max() < TOL, z


def test_gemm_dq16_rows_invariant(monkeypatch):
    """A row's dq16 value does not depend on the launch (the multi-GPU gather is bit-exact only if
    rank r's slab equals the same rows of the one-GPU call): slabs of 1000 / 512 / 128 rows starting
    at row 128 k, against the full 4096-row call, bit for bit."""
    monkeypatch.setenv("LAMM_GEMM_PATH", "dq16")
    M, N, K = 4096, 96, 2048
    A_q, B_q = random_case(ol.Q4_0, M, N, K, seed=99)
    full, _ = gpu_mul_mat(ol.Q4_0, A_q, B_q, M, N, K)
    arow = la.row_bytes(ol.Q4_0, K)
    for r0, rows in ((0, 1000), (1024, 512), (3968, 128)):
        part, _ = gpu_mul_mat(ol.Q4_0, A_q[r0 * arow:(r0 + rows) * arow], B_q, rows, N, K)
        assert np.array_equal(part, full[:, r0:r0 + rows]), (r0, rows)


DQ_RANGE_CASES = ["tiny_scales", "large_activations", "huge_activations", "large_weights", "tiny_activations",
                  "one_huge_column", "extremes"]


@pytest.mark.parametrize("case", DQ_RANGE_CASES)
def test_gemm_dq16_value_range(case, monkeypatch):
    """dq16 folds the block scales into f16 operands (weights pre-scaled by 2^8, activations by 2^4).
    Its range guard sends any tile whose scales leave f16's normal range, or whose
    f16 operands overflow, to exact int8 block dots -- so every case stays finite and within the bar,
    as the reference's exact kernels do (src/lamm_kernel_q8_0.hpp:50-117).
    tiny_scales: weight rows of magnitude 1e-5 (block scales ~1e-6); large_activations: |x| up to 3e4;
    huge_activations: |x| = 1e5 (d_b * b overflows f16); large_weights: |w| = 300 (q8_0 / q5_1
    d_a * 2^8 * q overflows); tiny_activations: |x| ~ 1e-6 (d_b subnormal); one_huge_column: one
    activation row of 1e5 among ordinary ones (only its tiles fall back); extremes: all-max / all-min
    quants (q4 nibbles 0 / 15, q8 -127 / 127)."""
    monkeypatch.setenv("LAMM_GEMM_PATH", "dq16")
    M, N, K = 256, 128, 1024
    rng = np.random.default_rng(3)
    a = rng.standard_normal((M, K), dtype=np.float32)
    b = rng.standard_normal((N, K), dtype=np.float32)
    if case == "tiny_scales":
        a *= 1e-5
    elif case == "large_activations":
        b *= 3e4 / np.abs(b).max()
    elif case == "huge_activations":
        b *= 1e5 / np.abs(b).max()
    elif case == "large_weights":
        a *= 300 / np.abs(a).max()
    elif case == "tiny_activations":
        b *= 1e-6
    elif case == "one_huge_column":
        b[70] *= 1e5 / np.abs(b[70]).max()
    else:
        a = np.where(np.arange(K) % 3 == 0, -1.0, 1.0).astype(np.float32) * np.ones((M, 1), np.float32)
        b = np.where(np.arange(K) % 2 == 0, 1.0, -1.0).astype(np.float32) * np.ones((N, 1), np.float32)
    for t in (ol.Q4_0, ol.Q5_1, ol.Q8_0):
        vt = la.vec_dot_type(t)
        A_q = ORACLE.quantize(t, a, ol.QUANT_REF)
        B_q = ORACLE.quantize(vt, b, ol.QUANT_AVX)
        assert la.gemm_engine(t, M, N, K) == "dq16"
        c, _ = gpu_mul_mat(t, A_q, B_q, M, N, K)
        ref = ORACLE.mul_mat(t, M, N, K, A_q, B_q)
        # q8_1 keeps s = d * sum(q) as fp16: beyond |x| ~ 2e3 the reference's own q5_1 sums overflow there
        fin = np.isfinite(ref)
        assert fin.all() or vt == ol.Q8_1, ol.NAMES[t]
        assert np.isfinite(c[fin]).all(), ol.NAMES[t]
        if fin.any():
            assert rel_err(c[fin], ref[fin], absdot(t, A_q, B_q, M, N, K)[fin]).max() < TOL, ol.NAMES[t]


@pytest.mark.parametrize("t", [ol.Q5_1, ol.Q8_0], ids=["q5_1", "q8_0"])
def test_gemm_default_engine_range(t):
    """The DEFAULT engine of a q5_1 / q8_0 prefill call (dq16 at config-4 sizes) with weights of
    magnitude 300 and activations of 1e5: finite and within the bar (its range guard's exact tiles)."""
    M, N, K = 4096, 512, 1024
    rng = np.random.default_rng(5)
    a = rng.standard_normal((M, K), dtype=np.float32)
    a *= 300 / np.abs(a).max()
    b = rng.standard_normal((N, K), dtype=np.float32)
    b[: N // 2] *= 1e5 / np.abs(b).max()
    vt = la.vec_dot_type(t)
    A_q = ORACLE.quantize(t, a, ol.QUANT_REF)
    B_q = ORACLE.quantize(vt, b, ol.QUANT_AVX)
    assert la.gemm_engine(t, M, N, K) == "dq16"
    c, _ = gpu_mul_mat(t, A_q, B_q, M, N, K)
    rows = np.random.default_rng(0).choice(M, 256, replace=False)
    arow = la.row_bytes(t, K)
    A_s = np.concatenate([A_q[r * arow:(r + 1) * arow] for r in rows])
    ref = ORACLE.mul_mat(t, len(rows), N, K, A_s, B_q)
    fin = np.isfinite(ref)   # (q8_1's fp16 s overflows in the reference itself beyond |x| ~ 2e3)
    assert fin.all() or t == ol.Q5_1
    assert fin.any() and np.isfinite(c[:, rows][fin]).all()
    assert rel_err(c[:, rows][fin], ref[fin], absdot(t, A_s, B_q, len(rows), N, K)[fin]).max() < TOL


@pytest.mark.parametrize("split", [1, 3, 8])
@pytest.mark.parametrize("t", FP6_TYPES, ids=[ol.NAMES[t] for t in FP6_TYPES])
def test_gemm_fp6_split_k(t, split, monkeypatch):
    """fp6 engine with K split over workgroups (LAMM_FP6_SPLIT; auto for grids < 256 tiles):
    uneven splits of 65 K-steps, partial tiles summed in split order by f6_reduce."""
    monkeypatch.setenv("LAMM_GEMM_PATH", "fp6")
    monkeypatch.setenv("LAMM_FP6_SPLIT", str(split))
    M, N, K = 300, 140, 4096 + 64
    A_q, B_q = random_case(t, M, N, K, seed=split)
    c, raw = gpu_mul_mat(t, A_q, B_q, M, N, K, ldc=M + 3)
    ref = ORACLE.mul_mat(t, M, N, K, A_q, B_q)
    assert rel_err(c, ref, absdot(t, A_q, B_q, M, N, K)).max() < TOL
    assert np.isnan(np.concatenate([raw[j * (M + 3) + M:(j + 1) * (M + 3)] for j in range(N)])).all()


FP6_KG_SHAPES = [(300, 140, 4096 + 64), (257, 129, 96), (33, 17, 1024), (130, 9, 8192 + 512), (64, 64, 64)]


@pytest.mark.parametrize("form", ["1", "1lds", "2"])
@pytest.mark.parametrize("t", FP6_TYPES, ids=[ol.NAMES[t] for t in FP6_TYPES])
@pytest.mark.parametrize("shape", FP6_KG_SHAPES, ids=[f"{m}x{n}x{k}" for m, n, k in FP6_KG_SHAPES])
def test_gemm_fp6_k_groups(t, shape, form, monkeypatch):
    """fp6 engine on 128x64 workgroup tiles whose waves split K into groups summed through LDS
    (LAMM_FP6_SUB=1: 4 groups of 64x64 waves streaming their own blocks, no barriers -- weights by
    LDS-DMA into per-wave rings, activations into VGPRs; "1lds": LAMM_FP6_AV=0, the barrier-staged
    LDS form; 2: 2 groups of 32x64 waves; automatic for grids
    of < 256 big tiles): K-step counts that leave groups with nothing in the last stage (65,
    2, 136 K-steps), tiles cut by M / N, C with a padded pitch."""
    monkeypatch.setenv("LAMM_GEMM_PATH", "fp6")
    monkeypatch.setenv("LAMM_FP6_SUB", form[0])
    if form == "1lds":
        monkeypatch.setenv("LAMM_FP6_AV", "0")
    M, N, K = shape
    A_q, B_q = random_case(t, M, N, K, seed=M + N + K + int(form[0]))
    c, raw = gpu_mul_mat(t, A_q, B_q, M, N, K, ldc=M + 3)
    ref = ORACLE.mul_mat(t, M, N, K, A_q, B_q)
    assert rel_err(c, ref, absdot(t, A_q, B_q, M, N, K)).max() < TOL
    assert np.isnan(np.concatenate([raw[j * (M + 3) + M:(j + 1) * (M + 3)] for j in range(N)])).all()


@pytest.mark.parametrize("split", [2, 3, 8])
@pytest.mark.parametrize("t", FP6_TYPES, ids=[ol.NAMES[t] for t in FP6_TYPES])
def test_gemm_fp6_split_k_fused_reduce_bitwise(t, split, monkeypatch):
    """The in-launch split-K fixup (each tile's last workgroup sums the partials) gives the SAME
    bits as the separate f6_reduce launch (both add in split order), over repeated calls (the
    tile counters must be left at zero) and a ragged grid; and matches the oracle."""
    monkeypatch.setenv("LAMM_GEMM_PATH", "fp6")
    monkeypatch.setenv("LAMM_FP6_SPLIT", str(split))
    M, N, K = 300, 140, 4096 + 64
    A_q, B_q = random_case(t, M, N, K, seed=40 + split)
    runs = []
    for fused in ("1", "1", "0", "1"):   # 1 = the in-launch fixup (an A/B switch), 0 = f6_reduce
        monkeypatch.setenv("LAMM_FP6_FUSED_REDUCE", fused)
        runs.append(gpu_mul_mat(t, A_q, B_q, M, N, K, ldc=M + 3)[0])
    for r in runs[1:]:
        assert np.array_equal(r.view(np.uint32), runs[0].view(np.uint32))
    ref = ORACLE.mul_mat(t, M, N, K, A_q, B_q)
    assert rel_err(runs[0], ref, absdot(t, A_q, B_q, M, N, K)).max() < TOL


@pytest.mark.parametrize("split", ["0", "4", "kg1", "kg2"])
@pytest.mark.parametrize("t", FP6_TYPES, ids=[ol.NAMES[t] for t in FP6_TYPES])
def test_gemm_fp6_batched_broadcast(t, split, monkeypatch):
    """fp6 engine with ggml batch dims: 2 weight slices broadcast over 4 activation slices
    (r2 = 2), the unique-A-slice prep indexing of lamm_gemm_fp6.hip; split-K partials
    indexed per slice; the K-group forms' tile order over slices."""
    monkeypatch.setenv("LAMM_GEMM_PATH", "fp6")
    if split.startswith("kg"):
        monkeypatch.setenv("LAMM_FP6_SUB", split[2:])
    else:
        monkeypatch.setenv("LAMM_FP6_SPLIT", split)
    M, N, K = 70, 20, 512
    kb = K // la.blck_size(t)
    vt = la.vec_dot_type(t)
    lda = pitch_blocks(t, kb)
    rng_seed = 11
    As = [random_case(t, M, N, K, seed=rng_seed + s)[0] for s in range(2)]
    Bs = [random_case(t, M, N, K, seed=rng_seed + 10 + s)[1] for s in range(4)]
    abytes = M * lda * la.type_size(t)
    A = dev_bytes(np.concatenate([pitched_A(t, a, M, kb, lda)[:abytes] for a in As]))
    bbytes = N * kb * la.type_size(vt)
    B = dev_bytes(np.concatenate([np.ascontiguousarray(b).view(np.uint8).reshape(-1)[:bbytes] for b in Bs]))
    C = torch.full((4 * N * M,), float("nan"), dtype=torch.float32, device="cuda")
    bt = la.Batch(2, 1, 4, 1, abytes, 2 * abytes, bbytes, 4 * bbytes, 4 * M * N, 4 * M * N * 4)
    la.mul_mat_torch(t, A, B, C, M, N, K, lda=lda, batch=bt)
    torch.cuda.synchronize()
    c = C.cpu().numpy().reshape(4, N, M)
    for z in range(4):
        a = As[z // 2]   # ggml broadcast: slice i12 uses weight slice i12 / r2
        ref = ORACLE.mul_mat(t, M, N, K, a, Bs[z])
        assert rel_err(c[z], ref, absdot(t, a, Bs[z], M, N, K)).max() < TOL, z


@pytest.mark.parametrize("t", ol.A_TYPES, ids=[ol.NAMES[t] for t in ol.A_TYPES])
def test_strided_operands(t):
    """A rows padded (lda > K/blck), B columns padded (ldb), C rows padded (ldc > M);
    bytes outside the logical C must stay untouched."""
    M, N, K = 37, 6, 1024
    kb = K // la.blck_size(t)
    A_q, B_q = random_case(t, M, N, K, seed=7)
    lda = pitch_blocks(t, kb + 5)
    c, raw = gpu_mul_mat(t, A_q, B_q, M, N, K, ldc=M + 11, lda=lda, ldb=kb + 3)
    ref = ORACLE.mul_mat(t, M, N, K, A_q, B_q)
    assert rel_err(c, ref, absdot(t, A_q, B_q, M, N, K)).max() < TOL
    gaps = np.concatenate([raw[j * (M + 11) + M:(j + 1) * (M + 11)] for j in range(N)])
    assert np.isnan(gaps).all(), "kernel wrote outside the logical C"


@pytest.mark.parametrize("t", ol.A_TYPES, ids=[ol.NAMES[t] for t in ol.A_TYPES])
def test_known_answer_constant(t):
    """src/la-benchmark-matmult.cpp:247-250: A=1, B=2 -> sum(C) = 2*K*M*N."""
    M, N, K = 48, 3, 4096
    vt = la.vec_dot_type(t)
    A_q = ORACLE.quantize(t, np.ones((M, K), np.float32))
    B_q = ORACLE.quantize(vt, np.full((N, K), 2.0, np.float32))
    c, _ = gpu_mul_mat(t, A_q, B_q, M, N, K)
    want = 2.0 * K * M * N
    assert abs(c.sum(dtype=np.float64) - want) / want < 1e-2


GEMV_FULL_TYPES = [ol.Q4_0, ol.Q4_1, ol.Q5_0, ol.Q5_1, ol.Q8_0, ol.Q2_K]


@pytest.mark.parametrize("t", GEMV_FULL_TYPES, ids=[ol.NAMES[t] for t in GEMV_FULL_TYPES])
def test_full_size_gemv_4096(t):
    """BASELINE config 2 shape (M=4096, N=1, K=4096) for Q4_0 and every config-4 format
    (src/la-benchmark-matmult.cpp:26-36): every row vs the oracle."""
    M, N, K = 4096, 1, 4096
    A_q, B_q = random_case(t, M, N, K, seed=42)
    c, _ = gpu_mul_mat(t, A_q, B_q, M, N, K)
    ref = ORACLE.mul_mat(t, M, N, K, A_q, B_q)
    assert rel_err(c, ref, absdot(t, A_q, B_q, M, N, K)).max() < TOL


SEG_KS = [4096 + 256, 11008, 12288, 12288 + 256]   # 2, 3 (ragged), 3 and 4 K-segments


@pytest.mark.parametrize("variant", ["0", "13"], ids=["segdma", "staged"])
@pytest.mark.parametrize("K", SEG_KS)
@pytest.mark.parametrize("t", ol.A_TYPES + ol.KQ_TYPES, ids=[ol.NAMES[t] for t in ol.A_TYPES + ol.KQ_TYPES])
def test_decode_multi_segment_k(t, K, variant, monkeypatch):
    """Single-column decode with K beyond one 4096-element segment (ffn_down's K = 11008):
    the multi-segment LDS-DMA kernel (default, 2-3 segments) and the LDS-staged segment
    kernel (LAMM_GEMV_VARIANT=13) against the oracle; ragged M (133 = 33 groups of 4 + 1)."""
    monkeypatch.setenv("LAMM_GEMV_VARIANT", variant)
    M, N = 133, 1
    if t in ol.KQ_TYPES:
        rng = np.random.default_rng(K + t)
        A_q = ol.random_kq_blocks(t, M, K, rng)
        B_q = ORACLE.quantize(ol.Q8_K, rng.standard_normal((N, K), dtype=np.float32))
    else:
        A_q, B_q = random_case(t, M, N, K, seed=K + t)
    c, _ = gpu_mul_mat(t, A_q, B_q, M, N, K)
    ref = ORACLE.mul_mat(t, M, N, K, A_q, B_q)
    assert rel_err(c, ref, absdot(t, A_q, B_q, M, N, K)).max() < TOL


def test_extreme_quants():
    """All-max / all-min quants (int8 -128/127 in B, nibble 0/15 in A): the exact
    int32 block dots must not saturate (v_dot4 without clamp)."""
    M, N, K = 16, 2, 4096
    t = ol.Q4_0
    A_q = ORACLE.quantize(t, np.full((M, K), -1.0, np.float32))
    A_q.reshape(M, -1)[:, :] = A_q.reshape(M, -1)
    B_q = ORACLE.quantize(ol.Q8_0, np.tile(np.where(np.arange(K) % 2 == 0, 1.0, -1.0).astype(np.float32), (N, 1)))
    c, _ = gpu_mul_mat(t, A_q, B_q, M, N, K)
    ref = ORACLE.mul_mat(t, M, N, K, A_q, B_q)
    assert np.allclose(c, ref, rtol=0, atol=1e-3 * np.abs(ref).max() + 1e-6)


DENSE_SHAPES = [(1, 1, 1), (37, 1, 3), (300, 2, 257), (33, 5, 1001), (70, 8, 4099), (19, 3, 9000), (5, 11, 2050)]


@pytest.mark.parametrize("t", [ol.F32, ol.F16], ids=["f32", "f16"])
@pytest.mark.parametrize("shape", DENSE_SHAPES, ids=[f"{m}x{n}x{k}" for m, n, k in DENSE_SHAPES])
def test_dense_rows_ragged_k(t, shape):
    """F32 / F16 rows of any length K (ggml allows it; lamm_gemv_dense.hip): the row pitch
    is padded to 16 bytes with NaN bit patterns, which the ragged-tail masking must keep out
    of the sums; K spans several activation segments for N up to 8 and beyond (grouped)."""
    M, N, K = shape
    rng = np.random.default_rng(M * 7 + N * 3 + K)
    vt = la.vec_dot_type(t)
    A_q = ORACLE.quantize(t, rng.standard_normal((M, K), dtype=np.float32))
    B_q = ORACLE.quantize(vt, rng.standard_normal((N, K), dtype=np.float32))
    eb = la.type_size(t)
    lda = pitch_blocks(t, K) + 16 // eb          # at least one padded 16-byte piece
    nan = np.array([0x7fc00000 if eb == 4 else 0x7e00], dtype=np.uint32 if eb == 4 else np.uint16)
    Ap = np.tile(nan, M * lda).view(np.uint8).reshape(M, lda * eb).copy()
    Ap[:, :K * eb] = A_q.reshape(M, K * eb)
    A = dev_bytes(np.concatenate([Ap.reshape(-1), np.zeros(64, np.uint8)]))
    B = dev_bytes(B_q)
    C = torch.full((N * M + 16,), float("nan"), dtype=torch.float32, device="cuda")
    la.mul_mat_torch(t, A, B, C, M, N, K, lda=lda)
    torch.cuda.synchronize()
    c = C.cpu().numpy()[:N * M].reshape(N, M)
    ref = ORACLE.mul_mat(t, M, N, K, A_q, B_q)
    assert np.isfinite(c).all()
    assert rel_err(c, ref, absdot(t, A_q, B_q, M, N, K)).max() < TOL


DGEMM_SHAPES = [(130, 129, 1000), (257, 300, 4096 + 8), (64, 33, 77), (128, 128, 128), (9, 700, 3)]


def _dense_case(t, M, N, K, seed, ldb_extra=0):
    rng = np.random.default_rng(seed)
    vt = la.vec_dot_type(t)
    A_q = ORACLE.quantize(t, rng.standard_normal((M, K), dtype=np.float32))
    B_q = ORACLE.quantize(vt, rng.standard_normal((N, K), dtype=np.float32))
    eb = la.type_size(t)
    lda = pitch_blocks(t, K) + 16 // eb
    nan = np.array([0x7fc00000 if eb == 4 else 0x7e00], dtype=np.uint32 if eb == 4 else np.uint16)
    Ap = np.tile(nan, M * lda).view(np.uint8).reshape(M, lda * eb).copy()
    Ap[:, :K * eb] = A_q.reshape(M, K * eb)
    ldb = K + ldb_extra
    Bp = np.tile(nan, N * ldb).view(np.uint8).reshape(N, ldb * eb).copy()
    Bp[:, :K * eb] = B_q.reshape(N, K * eb)
    return A_q, B_q, Ap, Bp, lda, ldb


@pytest.mark.parametrize("t", [ol.F32, ol.F16], ids=["f32", "f16"])
@pytest.mark.parametrize("shape", DGEMM_SHAPES, ids=[f"{m}x{n}x{k}" for m, n, k in DGEMM_SHAPES])
@pytest.mark.parametrize("bal", [True, False], ids=["b16", "bunaligned"])
def test_dense_gemm_vs_oracle(t, shape, bal):
    """F32 / F16 prefill GEMM on the matrix cores (lamm_gemm_dense.hip): ragged M / N / K
    against the 128x128 tile and 128-byte K-step, NaN row padding on both operands (masked),
    B rows 16-byte aligned (b128 loads) or not (element loads: F16 rows 2-byte aligned)."""
    M, N, K = shape
    eb = la.type_size(t)
    extra = (-K) % (16 // eb) if bal else (1 if (K * eb) % 16 == 0 else 0)
    A_q, B_q, Ap, Bp, lda, ldb = _dense_case(t, M, N, K, M * 7 + N * 3 + K, extra)
    assert ((ldb * eb) % 16 == 0) == bal
    A = dev_bytes(np.concatenate([Ap.reshape(-1), np.zeros(64, np.uint8)]))
    B = dev_bytes(np.concatenate([Bp.reshape(-1), np.zeros(64, np.uint8)]))
    C = torch.full((N * M + 16,), float("nan"), dtype=torch.float32, device="cuda")
    la.mul_mat_torch(t, A, B, C, M, N, K, lda=lda, ldb=ldb)
    torch.cuda.synchronize()
    c = C.cpu().numpy()[:N * M].reshape(N, M)
    ref = ORACLE.mul_mat(t, M, N, K, A_q, B_q)
    assert np.isfinite(c).all()
    assert rel_err(c, ref, absdot(t, A_q, B_q, M, N, K)).max() < TOL


@pytest.mark.parametrize("t", [ol.F32, ol.F16], ids=["f32", "f16"])
def test_dense_huge_row_pitch(t):
    """F32 / F16 prefill-sized call whose weight rows lie 2^24 + 64 bytes apart (a ggml view into a
    large tensor): 128 such rows are past the tiled GEMM's 32-bit buffer offsets, so the call runs on
    the grouped GEMV, which rebases per row -- within the bar, every row."""
    M, N, K = 9, 16, 256
    eb = la.type_size(t)
    lda = ((1 << 24) + 64) // eb
    rng = np.random.default_rng(3)
    A_q = ORACLE.quantize(t, rng.standard_normal((M, K), dtype=np.float32))
    B_q = ORACLE.quantize(t, rng.standard_normal((N, K), dtype=np.float32))
    A = torch.zeros(M * lda * eb + 64, dtype=torch.uint8, device="cuda")
    A[:M * lda * eb].view(M, lda * eb)[:, :K * eb] = \
        torch.from_numpy(np.ascontiguousarray(A_q).view(np.uint8).reshape(M, K * eb).copy()).cuda()
    B = dev_bytes(B_q)
    C = torch.full((N * M + 16,), float("nan"), dtype=torch.float32, device="cuda")
    la.mul_mat_torch(t, A, B, C, M, N, K, lda=lda)
    torch.cuda.synchronize()
    c = C.cpu().numpy()
    assert np.isnan(c[N * M:]).all()
    ref = ORACLE.mul_mat(t, M, N, K, A_q, B_q)
    assert rel_err(c[:N * M].reshape(N, M), ref, absdot(t, A_q, B_q, M, N, K)).max() < TOL


@pytest.mark.parametrize("t", [ol.F32, ol.F16], ids=["f32", "f16"])
def test_dense_gemm_batched_broadcast(t):
    """ggml batch dims on the dense GEMM: 2 weight slices broadcast over 2x3 activation slices
    (r2 = 1, r3 = 3 -- the GQA-style sharing of a KV-cache slice by several query heads)."""
    M, N, K = 70, 40, 200
    eb = la.type_size(t)
    cases = [_dense_case(t, M, N, K, 100 + s) for s in range(6)]
    lda, ldb = cases[0][4], cases[0][5]
    abytes, bbytes = M * lda * eb, N * ldb * eb
    A = dev_bytes(np.concatenate([cases[s][2].reshape(-1) for s in range(2)] + [np.zeros(64, np.uint8)]))
    B = dev_bytes(np.concatenate([cases[s][3].reshape(-1) for s in range(6)] + [np.zeros(64, np.uint8)]))
    C = torch.full((6 * N * M,), float("nan"), dtype=torch.float32, device="cuda")
    # ne02=2, ne03=1, ne12=2, ne13=3: slice (i12, i13) uses A slice (i12, i13 / 3)
    bt = la.Batch(2, 1, 2, 3, abytes, 2 * abytes, bbytes, 2 * bbytes, 4 * M * N, 4 * M * N * 2)
    la.mul_mat_torch(t, A, B, C, M, N, K, lda=lda, ldb=ldb, batch=bt)
    torch.cuda.synchronize()
    c = C.cpu().numpy().reshape(6, N, M)
    for z in range(6):
        a = cases[z % 2][0]
        ref = ORACLE.mul_mat(t, M, N, K, a, cases[z][1])
        assert rel_err(c[z], ref, absdot(t, a, cases[z][1], M, N, K)).max() < TOL, z


@pytest.mark.parametrize("t", [ol.Q4_0, ol.Q4_1, ol.Q5_0, ol.Q8_0, ol.F16], ids=["q4_0", "q4_1", "q5_0", "q8_0", "f16"])
def test_weights_stationary_matches_per_call(t, monkeypatch):
    """lamm_hip_weights_create / matmul_weights (packed prefill-GEMM weights kept on device)
    give the same bytes as the per-call path, on both the fp6 GEMM (forced, with a batched
    broadcast) and the GEMV; batch A dims other than the handle's are refused."""
    monkeypatch.setenv("LAMM_GEMM_PATH", "fp6")
    M, N, K = 300, 140, 1024
    eb = la.type_size(t)
    kb = K // la.blck_size(t)
    lda = pitch_blocks(t, kb)
    vt = la.vec_dot_type(t)
    As = [random_case(t, M, N, K, seed=40 + s)[0] for s in range(2)]
    Bs = [random_case(t, M, N, K, seed=50 + s)[1] for s in range(4)]
    abytes = M * lda * eb
    A = dev_bytes(np.concatenate([pitched_A(t, a, M, kb, lda)[:abytes] for a in As] + [np.zeros(64, np.uint8)]))
    bbytes = N * kb * la.type_size(vt)
    B = dev_bytes(np.concatenate([np.ascontiguousarray(b).view(np.uint8).reshape(-1)[:bbytes] for b in Bs]))
    bt = la.Batch(2, 1, 4, 1, abytes, 2 * abytes, bbytes, 4 * bbytes, 4 * M * N, 4 * M * N * 4)
    W = la.Weights(t, A, M, K, lda=lda, ne02=2, ne03=1, nba2=abytes, nba3=2 * abytes)
    assert (W.packed_bytes > 0) == (t in FP6_TYPES or t == ol.Q8_0)   # (q8_0: two code planes, round 6)
    for n in (N, 3):   # GEMM and GEMV
        C0 = torch.full((4 * n * M,), float("nan"), dtype=torch.float32, device="cuda")
        C1 = torch.full_like(C0, float("nan"))
        btn = la.Batch(2, 1, 4, 1, abytes, 2 * abytes, bbytes, 4 * bbytes, 4 * M * n, 4 * M * n * 4)
        la.mul_mat_torch(t, A, B, C0, M, n, K, lda=lda, batch=btn)
        W.matmul_torch(B, C1, n, batch=btn)
        torch.cuda.synchronize()
        assert torch.equal(C0, C1)
        c = C1.cpu().numpy().reshape(4, n, M)
        for z in range(4):
            Bz = np.ascontiguousarray(Bs[z]).view(np.uint8).reshape(-1)[:n * kb * la.type_size(vt)]
            ref = ORACLE.mul_mat(t, M, n, K, As[z // 2], Bz)
            assert rel_err(c[z], ref, absdot(t, As[z // 2], Bz, M, n, K)).max() < TOL
    bad = la.Batch(1, 1, 4, 1, abytes, abytes, bbytes, 4 * bbytes, 4 * M * N, 4 * M * N * 4)
    with pytest.raises(la.LammError):
        W.matmul_torch(B, C1, N, batch=bad)
    W.close()


@pytest.mark.parametrize("split", ["1", "3", "8"])
@pytest.mark.parametrize("t", [ol.F32, ol.F16], ids=["f32", "f16"])
def test_dense_gemm_split_k(t, split, monkeypatch):
    """Dense GEMM with K split over workgroups (LAMM_DENSE_SPLIT; auto under 256 tiles):
    uneven splits, ragged K tail in the last split, partials summed in split order."""
    monkeypatch.setenv("LAMM_DENSE_SPLIT", split)
    M, N, K = 200, 130, 2000 + 3
    A_q, B_q, Ap, Bp, lda, ldb = _dense_case(t, M, N, K, int(split) * 7 + t, (-K) % (16 // la.type_size(t)))
    A = dev_bytes(np.concatenate([Ap.reshape(-1), np.zeros(64, np.uint8)]))
    B = dev_bytes(np.concatenate([Bp.reshape(-1), np.zeros(64, np.uint8)]))
    C = torch.full((N * (M + 2) + 16,), float("nan"), dtype=torch.float32, device="cuda")
    la.mul_mat_torch(t, A, B, C, M, N, K, lda=lda, ldb=ldb, ldc=M + 2)
    torch.cuda.synchronize()
    c = C.cpu().numpy()
    got = np.stack([c[j * (M + 2):j * (M + 2) + M] for j in range(N)])
    ref = ORACLE.mul_mat(t, M, N, K, A_q, B_q)
    assert rel_err(got, ref, absdot(t, A_q, B_q, M, N, K)).max() < TOL
    assert np.isnan(np.concatenate([c[j * (M + 2) + M:(j + 1) * (M + 2)] for j in range(N)])).all()


def test_concurrent_streams_have_private_workspaces(monkeypatch):
    """Two GEMMs that need workspaces, issued back to back on two streams without
    synchronising in between: each (device, stream) has its own workspace, so neither
    overwrites the other's packed operands."""
    monkeypatch.setenv("LAMM_GEMM_PATH", "fp6")
    t, M, N, K = ol.Q4_0, 300, 100, 2048
    cases = [random_case(t, M, N, K, seed=90 + s) for s in range(2)]
    kb = K // 32
    streams = [torch.cuda.Stream() for _ in range(2)]
    outs = []
    for (A_q, B_q), st in zip(cases, streams):
        A = dev_bytes(pitched_A(t, A_q, M, kb, kb))
        B = dev_bytes(B_q)
        C = torch.full((N * M,), float("nan"), dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        with torch.cuda.stream(st):
            for _ in range(3):
                la.mul_mat_torch(t, A, B, C, M, N, K, stream=st.cuda_stream)
        outs.append((A, B, C))
    torch.cuda.synchronize()
    for (A_q, B_q), (_, _, C) in zip(cases, outs):
        ref = ORACLE.mul_mat(t, M, N, K, A_q, B_q)
        assert rel_err(C.cpu().numpy().reshape(N, M), ref, absdot(t, A_q, B_q, M, N, K)).max() < TOL


@pytest.mark.parametrize("engine", ["fp6", "i8", "kq"])
def test_weight_slice_beyond_2gib(engine, monkeypatch):
    """One weight slice of ~2.3 GB (1M rows): the prep passes address rows through buffer
    resources based at the rows they read, so rows past 2 GiB are not clipped to zeros.
    Checks the first and last 64 rows of C against the oracle."""
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    t = ol.Q4_K if engine == "kq" else ol.Q4_0
    if engine != "kq":
        monkeypatch.setenv("LAMM_GEMM_PATH", engine)
    M, N, K = 1_000_000, 16, 4096
    gen = torch.Generator(device="cuda")
    gen.manual_seed(5)
    fmt = ol.NAMES[t]
    A, arow = bench.make_weights(torch, la, fmt, 1, M, K, gen)
    assert M * arow > 2 ** 31
    rng = np.random.default_rng(1)
    vt = la.vec_dot_type(t)
    B_q = ORACLE.quantize(vt, rng.standard_normal((N, K), dtype=np.float32),
                          ol.QUANT_AVX if vt == ol.Q8_0 else ol.QUANT_REF)
    B = dev_bytes(B_q)
    C = torch.full((N * M,), float("nan"), dtype=torch.float32, device="cuda")
    la.mul_mat_torch(t, A, B, C, M, N, K)
    torch.cuda.synchronize()
    c = C.view(N, M)
    for r0 in (0, M - 64):
        a_rows = A[r0 * arow:(r0 + 64) * arow].cpu().numpy()
        ref = ORACLE.mul_mat(t, 64, N, K, a_rows, B_q)
        got = c[:, r0:r0 + 64].cpu().numpy()
        assert rel_err(got, ref, absdot(t, a_rows, B_q, 64, N, K)).max() < TOL, r0
    del A, C
    torch.cuda.empty_cache()


SPLIT_TYPES = [ol.Q4_0, ol.Q5_1, ol.Q8_0, ol.Q4_K, ol.Q6_K, ol.Q2_K]


@pytest.mark.parametrize("split", ["0", "1", "3", "16"])
@pytest.mark.parametrize("t", SPLIT_TYPES, ids=[ol.NAMES[t] for t in SPLIT_TYPES])
def test_gemm_split_k_i8_and_superblock(t, split, monkeypatch):
    """K-split of the MFMA-i8 (LAMM_I8_SPLIT) and super-block (LAMM_KQ_SPLIT) GEMMs, on a
    la-benchmark-matmult-like shape (K = 11008, the reference's default; one 64-row tile
    column so the auto policy splits): uneven splits, partials summed in split order, padded
    C pitch left untouched."""
    monkeypatch.setenv("LAMM_GEMM_PATH", "i8")
    monkeypatch.setenv("LAMM_I8_SPLIT", split)
    monkeypatch.setenv("LAMM_KQ_SPLIT", split)
    M, N, K = 200, 130, 11008
    rng = np.random.default_rng(int(split) * 31 + t)
    if t in ol.KQ_TYPES:
        A_q = ol.random_kq_blocks(t, M, K, rng)
    else:
        A_q = ORACLE.quantize(t, rng.standard_normal((M, K), dtype=np.float32))
    vt = ORACLE.vec_dot_type(t)
    B_q = ORACLE.quantize(vt, rng.standard_normal((N, K), dtype=np.float32),
                          ol.QUANT_AVX if vt in (ol.Q8_0, ol.Q8_1) else 0)
    kb = K // la.blck_size(t)
    c, raw = gpu_mul_mat(t, A_q, B_q, M, N, K, lda=pitch_blocks(t, kb), ldc=M + 3)
    ref = ORACLE.mul_mat(t, M, N, K, A_q, B_q)
    assert rel_err(c, ref, absdot(t, A_q, B_q, M, N, K)).max() < TOL
    assert np.isnan(np.concatenate([raw[j * (M + 3) + M:(j + 1) * (M + 3)] for j in range(N)])).all()


FUSED_TYPES = [ol.Q4_0, ol.Q4_1, ol.Q5_0, ol.Q5_1, ol.Q8_0]
FUSED_SHAPES = [(64, 1, 4096), (200, 3, 11008), (37, 8, 96), (130, 5, 4160), (64, 2, 8192 + 512)]


@pytest.mark.parametrize("t", FUSED_TYPES, ids=[ol.NAMES[t] for t in FUSED_TYPES])
@pytest.mark.parametrize("shape", FUSED_SHAPES, ids=[f"{m}x{n}x{k}" for m, n, k in FUSED_SHAPES])
def test_decode_gemv_f32_activations_fused(t, shape):
    """F32 activations straight into the decode GEMV (ggml's INIT quantization fused into the
    launch): C must be BIT-identical to lamm_hip_quantize(flavour 1) + matmul on the same
    rows -- every GEMV kernel (stream, LDS-DMA, multi-segment, segmented) -- and match the
    oracle on the reference's quantized bytes."""
    M, N, K = shape
    rng = np.random.default_rng(M + 7 * N + K + t)
    A_q = ORACLE.quantize(t, rng.standard_normal((M, K), dtype=np.float32))
    x = rng.standard_normal((N, K), dtype=np.float32)
    x[0, :32] = 0.0                                   # an all-zero block (d = 0)
    ldx = K + 4                                        # padded F32 rows (NaN padding)
    xp = np.full((N, ldx), np.nan, np.float32)
    xp[:, :K] = x
    kb = K // 32
    lda = pitch_blocks(t, kb)
    dA = dev_bytes(pitched_A(t, A_q, M, kb, lda))
    dx = torch.from_numpy(xp.reshape(-1)).cuda()
    s = torch.cuda.current_stream().cuda_stream
    c1 = torch.full((N * M,), np.nan, dtype=torch.float32, device="cuda")
    la.matmul(la.Matrix(dA.data_ptr(), t, M, kb, lda), la.Matrix(dx.data_ptr(), la.F32, K, N, ldx),
              la.Matrix(c1.data_ptr(), la.F32, M, N, M), s)
    vt = ORACLE.vec_dot_type(t)
    dq = torch.zeros(N * la.row_bytes(vt, K) + 64, dtype=torch.uint8, device="cuda")
    la.quantize_torch(vt, dx.view(N, ldx)[:, :K], dq, flavour=1)
    c2 = torch.full((N * M,), np.nan, dtype=torch.float32, device="cuda")
    la.matmul(la.Matrix(dA.data_ptr(), t, M, kb, lda), la.Matrix(dq.data_ptr(), vt, kb, N, kb),
              la.Matrix(c2.data_ptr(), la.F32, M, N, M), s)
    torch.cuda.synchronize()
    a, b = c1.cpu().numpy(), c2.cpu().numpy()
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    B_q = ORACLE.quantize(vt, x, ol.QUANT_AVX)
    assert np.array_equal(dq.cpu().numpy()[:B_q.size], B_q)
    ref = ORACLE.mul_mat(t, M, N, K, A_q, B_q)
    assert rel_err(a.reshape(N, M), ref, absdot(t, A_q, B_q, M, N, K)).max() < TOL


GEMM_F32_CASES = [(ol.Q4_0, "fp6"), (ol.Q4_0, "i8"), (ol.Q4_1, "fp6"), (ol.Q4_1, "i8"), (ol.Q5_0, "fp6"),
                  (ol.Q5_0, "i8"), (ol.Q5_1, "default"), (ol.Q8_0, "default")]


@pytest.mark.parametrize("t,path", GEMM_F32_CASES, ids=[f"{ol.NAMES[t]}-{p}" for t, p in GEMM_F32_CASES])
@pytest.mark.parametrize("N", [9, 140])
def test_gemm_f32_activations(t, path, N, monkeypatch):
    """F32 B for N > 8 (ggml's INIT quantization on the device): quantized inside the fp6 and
    i8 engines' activation preps -- C must be BIT-identical to lamm_hip_quantize(flavour 1) +
    matmul either way, and match the oracle."""
    if path != "default":
        monkeypatch.setenv("LAMM_GEMM_PATH", path)
    M, K = 300, 4096 + 64
    rng = np.random.default_rng(N + t)
    A_q = ORACLE.quantize(t, rng.standard_normal((M, K), dtype=np.float32))
    x = rng.standard_normal((N, K), dtype=np.float32)
    x[1, 64:96] = 0.0                                  # an all-zero block (d = 0)
    ldx = K + 4 if N > 100 else K + 1                  # NaN-padded rows; odd pitch: 4-byte aligned only
    xp = np.full((N, ldx), np.nan, np.float32)
    xp[:, :K] = x
    kb = K // 32
    lda = pitch_blocks(t, kb)
    dA = dev_bytes(pitched_A(t, A_q, M, kb, lda))
    dx = torch.from_numpy(xp.reshape(-1)).cuda()
    s = torch.cuda.current_stream().cuda_stream
    c1 = torch.full((N * M,), np.nan, dtype=torch.float32, device="cuda")
    la.matmul(la.Matrix(dA.data_ptr(), t, M, kb, lda), la.Matrix(dx.data_ptr(), la.F32, K, N, ldx),
              la.Matrix(c1.data_ptr(), la.F32, M, N, M), s)
    vt = ORACLE.vec_dot_type(t)
    dq = torch.zeros(N * la.row_bytes(vt, K) + 64, dtype=torch.uint8, device="cuda")
    la.quantize_torch(vt, dx.view(N, ldx)[:, :K].contiguous(), dq, flavour=1)   # the quantizer wants 16-byte rows
    c2 = torch.full((N * M,), np.nan, dtype=torch.float32, device="cuda")
    la.matmul(la.Matrix(dA.data_ptr(), t, M, kb, lda), la.Matrix(dq.data_ptr(), vt, kb, N, kb),
              la.Matrix(c2.data_ptr(), la.F32, M, N, M), s)
    torch.cuda.synchronize()
    a, b = c1.cpu().numpy(), c2.cpu().numpy()
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    B_q = ORACLE.quantize(vt, x, ol.QUANT_AVX)
    ref = ORACLE.mul_mat(t, M, N, K, A_q, B_q)
    assert rel_err(a.reshape(N, M), ref, absdot(t, A_q, B_q, M, N, K)).max() < TOL


# ---------------------------------------------------------------- BASELINE config 3, full size
def _config3_operands(seed, slices):
    """Q4_0 A (4096 x 4096, `slices` distinct slices) quantized from N(0,1) by the oracle's
    reference quantizer, B = 512 q8_0 rows (AVX2 flavour, ggml's INIT on x86)."""
    M, N, K = 4096, 512, 4096
    rng = np.random.default_rng(seed)
    As = [ORACLE.quantize(ol.Q4_0, rng.standard_normal((M, K), dtype=np.float32)) for _ in range(slices)]
    Bs = [ORACLE.quantize(ol.Q8_0, rng.standard_normal((N, K), dtype=np.float32), ol.QUANT_AVX)
          for _ in range(slices)]
    return As, Bs


def _config3_check(c, A_q, B_q, rows):
    """c: [N][M] GPU result; compare the sampled rows (all 512 columns) with the oracle."""
    M, N, K = 4096, 512, 4096
    arow = la.row_bytes(ol.Q4_0, K)
    a = np.concatenate([A_q[r * arow:(r + 1) * arow] for r in rows])
    ref = ORACLE.mul_mat(ol.Q4_0, len(rows), N, K, a, B_q)
    err = rel_err(c[:, rows], ref, absdot(ol.Q4_0, a, B_q, len(rows), N, K)).max()
    assert np.isfinite(c).all()
    return err


CONFIG3_ROWS = np.unique(np.concatenate([np.arange(0, 4096, 16), [1, 127, 128, 255, 256, 2047, 2048, 4095]]))


@pytest.mark.parametrize("path", ["stationary_auto", "stationary_fp6_split_k", "stationary_fp6_kgroups2",
                                  "per_call_default", "per_call_fp6", "per_call_i8", "per_call_dq16"])
def test_config3_full_size_gemm(path, monkeypatch):
    """BASELINE config 3 at its real size: Q4_0 x Q8_0 M=4096 N=512 K=4096, one slice.
    Paths: the weight-stationary handle (the ggml boundary's and bench.py's; fp6 engine, by
    default 256 128x64 tiles with 4 K-groups each, or forced: K split over the 64 256x128 tiles,
    2 K-groups), the per-call API's default engine, and the exact engines and the dequantizing f16
    engine forced per call.  >= 256 sampled rows x all 512 columns vs the oracle."""
    M, N, K = 4096, 512, 4096
    (A_q,), (B_q,) = _config3_operands(2024, 1)
    if path in ("per_call_fp6", "per_call_i8", "per_call_dq16"):
        monkeypatch.setenv("LAMM_GEMM_PATH", path.rsplit("_", 1)[1])
    if path == "stationary_fp6_split_k":
        monkeypatch.setenv("LAMM_FP6_SUB", "0")
    if path == "stationary_fp6_kgroups2":
        monkeypatch.setenv("LAMM_FP6_SUB", "2")
    A = dev_bytes(np.concatenate([A_q, np.zeros(64, np.uint8)]))
    B = dev_bytes(B_q)
    C = torch.full((N * M,), float("nan"), dtype=torch.float32, device="cuda")
    if path.startswith("stationary"):
        assert la.gemm_engine("q4_0", M, N, K, 1, stationary=True) == "fp6"
        W = la.Weights(ol.Q4_0, A, M, K)
        W.matmul_torch(B, C, N)
        torch.cuda.synchronize()
        W.close()
    else:
        la.mul_mat_torch(ol.Q4_0, A, B, C, M, N, K)
        torch.cuda.synchronize()
    err = _config3_check(C.cpu().numpy().reshape(N, M), A_q, B_q, CONFIG3_ROWS)
    print(f"config 3 {path}: max rel err {err:.2e} over {len(CONFIG3_ROWS)} rows x {N}")
    assert err < TOL


@pytest.mark.parametrize("act", ["q8", "f32"])
def test_config3_repeated_calls_fresh_activations(act, monkeypatch):
    """Config 3, three calls with DIFFERENT activations into the same per-stream workspace (B1,
    B2, B1): the packed activation tiles the prep writes there and the main kernel reads back
    must never be served stale from an earlier call.  q8 rows through the weight-stationary
    handle, or F32 rows (quantized on the device) through the per-call API."""
    M, N, K = 4096, 512, 4096
    rng = np.random.default_rng(77)
    (A_q,), _ = _config3_operands(2025, 1)
    xs = [rng.standard_normal((N, K), dtype=np.float32) for _ in range(2)]
    Bq = [ORACLE.quantize(ol.Q8_0, x, ol.QUANT_AVX) for x in xs]
    A = dev_bytes(np.concatenate([A_q, np.zeros(64, np.uint8)]))
    W = la.Weights(ol.Q4_0, A, M, K)
    rows = CONFIG3_ROWS[::2]
    s = torch.cuda.current_stream().cuda_stream
    monkeypatch.setenv("LAMM_GEMM_PATH", "fp6")   # the F32 calls go through the per-call API
    for k in (0, 1, 0):
        C = torch.full((N * M,), float("nan"), dtype=torch.float32, device="cuda")
        if act == "q8":
            W.matmul_torch(dev_bytes(Bq[k]), C, N)
        else:
            X = torch.from_numpy(xs[k]).cuda()
            la.matmul(la.Matrix(A.data_ptr(), ol.Q4_0, M, K // 32, K // 32), la.Matrix(X.data_ptr(), la.F32, K, N, K),
                      la.Matrix(C.data_ptr(), la.F32, M, N, M), s)
        torch.cuda.synchronize()
        err = _config3_check(C.cpu().numpy().reshape(N, M), A_q, Bq[k], rows)
        assert err < TOL, (k, err)
    W.close()


@pytest.mark.parametrize("engine", ["fp6", "dq16"])
def test_config3_four_slice_batched_launch(engine, monkeypatch):
    """The 4-slice batched launch bench.py times (ne02 = ne12 = 4, stationary weights; the default
    fp6 engine with 256 tiles, or the dequantizing f16 engine forced, 1024 tiles): every slice's
    sampled rows x all columns vs the oracle."""
    if engine == "dq16":
        monkeypatch.setenv("LAMM_GEMM_PATH", "dq16")
    M, N, K = 4096, 512, 4096
    As, Bs = _config3_operands(77, 4)
    arow, brow = la.row_bytes(ol.Q4_0, K), la.row_bytes(ol.Q8_0, K)
    A = dev_bytes(np.concatenate(As + [np.zeros(64, np.uint8)]))
    B = dev_bytes(np.concatenate(Bs))
    C = torch.full((4 * N * M,), float("nan"), dtype=torch.float32, device="cuda")
    bt = la.Batch(4, 1, 4, 1, M * arow, 4 * M * arow, N * brow, 4 * N * brow, 4 * M * N, 16 * M * N)
    assert la.gemm_engine("q4_0", M, N, K, 4, stationary=True) == engine
    W = la.Weights(ol.Q4_0, A, M, K, ne02=4, ne03=1, nba2=M * arow, nba3=4 * M * arow)
    W.matmul_torch(B, C, N, batch=bt)
    torch.cuda.synchronize()
    W.close()
    c = C.cpu().numpy().reshape(4, N, M)
    rows = CONFIG3_ROWS[::4]
    for z in range(4):
        err = _config3_check(c[z], As[z], Bs[z], rows)
        assert err < TOL, (z, err)


# ---------------------------------------------------------------- row-per-wave decode GEMV
RPW_TYPES = [ol.Q4_0, ol.Q4_1, ol.Q5_0, ol.Q5_1, ol.Q8_0]
RPW_SHAPES = [(1, 1, 32), (5, 1, 96), (67, 2, 512), (130, 1, 4096), (33, 2, 4096 + 256), (9, 1, 11008),
              (257, 1, 8192 + 32), (133, 1, 10272), (70, 1, 12288), (4096, 1, 11008)]


@pytest.mark.parametrize("rows", ["4", "8", "16"])
@pytest.mark.parametrize("t", RPW_TYPES, ids=[ol.NAMES[t] for t in RPW_TYPES])
@pytest.mark.parametrize("shape", RPW_SHAPES, ids=[f"{m}x{n}x{k}" for m, n, k in RPW_SHAPES])
def test_gemv_row_per_wave(t, shape, rows, monkeypatch):
    """lamm_gemv_rpw.hip (LAMM_GEMV_RPW = waves per workgroup, 8 at most past K = 4096): ragged
    M / K, one and two columns, q8 activations and F32 activations (INIT fused, must equal
    quantize + matmul).  One column, K = 4096 and 8 waves: the flat kernel (2 runs of 64 blocks per
    row)."""
    monkeypatch.setenv("LAMM_GEMV_RPW", rows)
    M, N, K = shape
    A_q, B_q = random_case(t, M, N, K, seed=M * 7 + K + int(rows))
    got, _ = gpu_mul_mat(t, A_q, B_q, M, N, K)
    ref = ORACLE.mul_mat(t, M, N, K, A_q, B_q)
    assert rel_err(got, ref, absdot(t, A_q, B_q, M, N, K)).max() < TOL
    # F32 activations: the kernel quantizes them (AVX2 flavour) -> same C as the q8 path
    rng = np.random.default_rng(M + K)
    x = rng.standard_normal((N, K), dtype=np.float32)
    vt = la.vec_dot_type(t)
    Bx = ORACLE.quantize(vt, x, ol.QUANT_AVX)
    kb = K // 32
    lda = pitch_blocks(t, kb)
    A = dev_bytes(pitched_A(t, A_q, M, kb, lda))
    X = torch.from_numpy(x).cuda()
    C = torch.full((N * M,), float("nan"), dtype=torch.float32, device="cuda")
    la.matmul(la.Matrix(A.data_ptr(), t, M, kb, lda), la.Matrix(X.data_ptr(), la.F32, K, N, K),
              la.Matrix(C.data_ptr(), la.F32, M, N, M), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    want, _ = gpu_mul_mat(t, A_q, Bx, M, N, K)
    np.testing.assert_array_equal(C.cpu().numpy().reshape(N, M), want)


def test_gemv_row_per_wave_batched_broadcast(monkeypatch):
    """Batch slices (ne02 = 2 broadcast over ne12 = 4) through the row-per-wave kernel."""
    monkeypatch.setenv("LAMM_GEMV_RPW", "16")
    t, M, N, K = ol.Q4_0, 100, 1, 1024
    kb = K // 32
    As = [random_case(t, M, N, K, seed=200 + s)[0] for s in range(2)]
    Bs = [random_case(t, M, N, K, seed=210 + s)[1] for s in range(4)]
    abytes, bbytes = M * kb * 18, N * kb * 34
    A = dev_bytes(np.concatenate(As + [np.zeros(64, np.uint8)]))
    B = dev_bytes(np.concatenate(Bs))
    C = torch.full((4 * N * M,), float("nan"), dtype=torch.float32, device="cuda")
    bt = la.Batch(2, 1, 4, 1, abytes, 2 * abytes, bbytes, 4 * bbytes, 4 * M * N, 16 * M * N)
    la.mul_mat_torch(t, A, B, C, M, N, K, batch=bt)
    torch.cuda.synchronize()
    c = C.cpu().numpy().reshape(4, N, M)
    for z in range(4):
        ref = ORACLE.mul_mat(t, M, N, K, As[z // 2], Bs[z])
        assert rel_err(c[z], ref, absdot(t, As[z // 2], Bs[z], M, N, K)).max() < TOL, z


@pytest.mark.parametrize("t", RPW_TYPES, ids=[ol.NAMES[t] for t in RPW_TYPES])
def test_gemv_row_slab_invariance(t):
    """A row's value does not depend on the launch it is in: the 4096 x 4096 decode GEMV (flat
    kernel, 8 waves) against row slabs of it as `bench.py --gpus N` shards them (2048 rows: flat;
    1024 / 512 / 1000: the row-per-wave kernel with 4 waves) and one column against the same
    column inside a two-column call -- bit-identical, as the multi-GPU gather check requires."""
    M, K = 4096, 4096
    A_q, B_q = random_case(t, M, 2, K, seed=9100 + t)
    rows_q = np.ascontiguousarray(A_q).reshape(M, -1)
    b1 = np.ascontiguousarray(B_q).reshape(2, -1)[:1]
    full, _ = gpu_mul_mat(t, rows_q, b1, M, 1, K)
    full = np.asarray(full).reshape(-1)
    for r0, rows in ((0, 2048), (2048, 1024), (3584, 512), (1000, 1000)):
        slab, _ = gpu_mul_mat(t, np.ascontiguousarray(rows_q[r0:r0 + rows]), b1, rows, 1, K)
        np.testing.assert_array_equal(np.asarray(slab).reshape(-1), full[r0:r0 + rows], err_msg=f"rows {r0}+{rows}")
    two, _ = gpu_mul_mat(t, rows_q, B_q, M, 2, K)
    np.testing.assert_array_equal(np.asarray(two).reshape(2, M)[0], full)


# ---------------------------------------------------------------- BASELINE config 4, full size
CONFIG4_TYPES = [ol.Q4_1, ol.Q5_0, ol.Q5_1, ol.Q8_0, ol.Q2_K]   # src/la-benchmark-matmult.cpp:26-36
_CONFIG4_CACHE = {}


def _config4_operands(t):
    """A = t-quantized N(0,1) 4096 x 4096 (the oracle's reference quantizer), B = 512 rows of
    vec_dot_type(t) (AVX2 flavour for q8_0 / q8_1, as ggml's INIT on x86)."""
    if t not in _CONFIG4_CACHE:
        M, N, K = 4096, 512, 4096
        rng = np.random.default_rng(4000 + t)
        vt = la.vec_dot_type(t)
        A_q = ORACLE.quantize(t, rng.standard_normal((M, K), dtype=np.float32))
        B_q = ORACLE.quantize(vt, rng.standard_normal((N, K), dtype=np.float32),
                              ol.QUANT_AVX if vt in (ol.Q8_0, ol.Q8_1) else ol.QUANT_REF)
        _CONFIG4_CACHE.clear()
        _CONFIG4_CACHE[t] = (A_q, B_q)
    return _CONFIG4_CACHE[t]


@pytest.mark.parametrize("mode", ["stationary", "per_call"])
@pytest.mark.parametrize("t", CONFIG4_TYPES, ids=[ol.NAMES[t] for t in CONFIG4_TYPES])
def test_config4_full_size_gemm(t, mode):
    """BASELINE config 4 at its real size: every sweep format at M=4096 N=512 K=4096 on its
    default prefill engine (q4_1 / q5_0: fp6; q5_1: fp6 with prepared weights, dq16 per call; q8_0:
    dq16, range-guarded; q2_K: the super-block engine), through the weight-stationary handle (the
    ggml boundary's and bench.py's path) and the per-call API.  >= 256 sampled rows x all 512
    columns vs the oracle."""
    M, N, K = 4096, 512, 4096
    A_q, B_q = _config4_operands(t)
    A = dev_bytes(np.concatenate([A_q, np.zeros(64, np.uint8)]))
    B = dev_bytes(B_q)
    C = torch.full((N * M,), float("nan"), dtype=torch.float32, device="cuda")
    if mode == "stationary":
        W = la.Weights(t, A, M, K)
        W.matmul_torch(B, C, N)
        torch.cuda.synchronize()
        W.close()
    else:
        la.mul_mat_torch(t, A, B, C, M, N, K)
        torch.cuda.synchronize()
    c = C.cpu().numpy().reshape(N, M)
    assert np.isfinite(c).all()
    arow = la.row_bytes(t, K)
    rows = CONFIG3_ROWS
    a = np.concatenate([A_q[r * arow:(r + 1) * arow] for r in rows])
    ref = ORACLE.mul_mat(t, len(rows), N, K, a, B_q)
    err = rel_err(c[:, rows], ref, absdot(t, a, B_q, len(rows), N, K)).max()
    print(f"config 4 {ol.NAMES[t]} {mode} [{la.gemm_engine(t, M, N, K, 1, stationary=mode == 'stationary')}]: "
          f"max rel err {err:.2e} over {len(rows)} rows x {N}")
    assert err < TOL


# ---------------------------------------------------------------- BASELINE config 1
def test_config1_f32_512_cube():
    """BASELINE config 1 (la-benchmark-matmult F32 M=N=K=512, src/la-benchmark-matmult.cpp:257-276)
    on the GPU's F32 path (the dense prefill GEMM): every output vs the oracle's F32 dot."""
    M = N = K = 512
    rng = np.random.default_rng(512)
    a = rng.standard_normal((M, K), dtype=np.float32)
    b = rng.standard_normal((N, K), dtype=np.float32)
    c, _ = gpu_mul_mat(ol.F32, a.view(np.uint8), b.view(np.uint8), M, N, K)
    ref = ORACLE.mul_mat(ol.F32, M, N, K, a.view(np.uint8), b.view(np.uint8))
    absd = np.abs(b.astype(np.float64)) @ np.abs(a.astype(np.float64)).T
    assert rel_err(c, ref, absd).max() < TOL


# ---------------------------------------------------------------- q2_K single-column decode
Q2K_SHAPES = [(1, 256), (9, 4096), (133, 4352), (64, 8192), (37, 11008), (4096, 4096), (70, 12288)]


@pytest.mark.parametrize("t", [ol.Q2_K, ol.Q4_K, ol.Q5_K, ol.Q6_K], ids=["q2_k", "q4_k", "q5_k", "q6_k"])
@pytest.mark.parametrize("shape", Q2K_SHAPES + [(32000, 1024)], ids=[f"{m}x1x{k}" for m, k in Q2K_SHAPES + [(32000, 1024)]])
def test_gemv_kq_row_per_wave(t, shape):
    """lamm_gemv_rpw.hip's k-quant kernel (one column, up to 48 super-blocks per row): lanes on
    quarter super-blocks, the quarters' integer sums combined in the quad (exact), one float
    epilogue per super-block as the reference's ggml_vec_dot_q{2,4,5,6}_K_q8_K; ragged M, K from one
    to 48 super-blocks, against the oracle.  q6_K (210-byte, 2-byte aligned super-blocks) takes every
    row count: a Q4_0 model's 32000-row output.weight (LC/llama.cpp:11731-11742)."""
    M, K = shape
    if M == 32000 and t != ol.Q6_K:
        pytest.skip("the long grid is q6_K's case (output.weight)")
    rng = np.random.default_rng(M * 31 + K + t)
    A_q = ol.random_kq_blocks(t, M, K, rng)
    B_q = ORACLE.quantize(ol.Q8_K, rng.standard_normal((1, K), dtype=np.float32))
    c, _ = gpu_mul_mat(t, A_q, B_q, M, 1, K)
    ref = ORACLE.mul_mat(t, M, 1, K, A_q, B_q)
    assert rel_err(c, ref, absdot(t, A_q, B_q, M, 1, K)).max() < TOL
