"""q5_1 prefill on the block-scaled fp6 engine (lamm_gemm_fp6.hip F6<kQ5_1>): its quants are coded as
q - 16 (exact in e2m3) and the shift rides on the affine term in the m * s MFMA's spare k slots:
sum_b (m_a s_b + 16 d_a (s_b + r_b)), r_b the activation prep's residual of the block's rounded s_b
(round 6, lamm_gemm_fp6.hip SH16), so the shift's share is 16 d_a d_b sum q_b as in the reference.  Only weight-stationary calls take it (lamm_hip_weights_create packs and range-
checks the weights once); a tensor with a block scale past 2047 (32 d leaves f16; round 6) keeps no packed form
and runs on the range-guarded dq16 engine.  Checked against the oracle (the reference's lamm q5_1
block kernel, src/lamm_kernel_q5_1.hpp) at the usual bar."""
import numpy as np
import pytest

from conftest import rel_err
import oracle_lib as ol

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
import lamm_amd as la  # noqa: E402
from test_gpu_parity import TOL, absdot, dev_bytes, pitch_blocks, pitched_A  # noqa: E402

ORACLE = ol.Oracle()
T = ol.Q5_1
SHAPES = [(33, 17, 1024), (130, 9, 8192 + 512), (257, 129, 4096 + 64), (300, 40, 96), (4096, 512, 4096)]


def stationary(A_q, B_q, M, N, K):
    kb = K // 32
    lda = pitch_blocks(T, kb)
    A = dev_bytes(pitched_A(T, A_q, M, kb, lda))
    B = dev_bytes(B_q)
    C = torch.full((N * M + 16,), float("nan"), dtype=torch.float32, device="cuda")
    W = la.Weights(T, A, M, K, lda=lda)
    packed = W.packed_bytes
    W.matmul_torch(B, C, N)
    torch.cuda.synchronize()
    W.close()
    c = C.cpu().numpy()
    assert np.isnan(c[N * M:]).all()
    return c[:N * M].reshape(N, M), packed


def check(c, A_q, B_q, M, N, K, rows):
    kb = K // 32
    arow = kb * la.type_size(T)
    A_s = np.ascontiguousarray(A_q).reshape(M, arow)[rows].reshape(-1)
    ref = ORACLE.mul_mat(T, len(rows), N, K, A_s, B_q)
    assert np.isfinite(c).all()
    return rel_err(c[:, rows], ref, absdot(T, A_s, B_q, len(rows), N, K)).max()


@pytest.mark.parametrize("shape", SHAPES, ids=[f"{m}x{n}x{k}" for m, n, k in SHAPES])
def test_q5_1_fp6_stationary_vs_oracle(shape, monkeypatch):
    M, N, K = shape
    if M * N < 4096 * 512:   # small calls: the fp6 engine forced (by default they take the i8 engine)
        monkeypatch.setenv("LAMM_GEMM_PATH", "fp6")
    assert la.gemm_engine(T, M, N, K, 1, stationary=True) == "fp6"
    rng = np.random.default_rng(M + N + K)
    a = rng.standard_normal((M, K), dtype=np.float32)
    a[:, :64] += 3.0   # blocks with a large min as well as centred ones
    A_q = ORACLE.quantize(T, a, ol.QUANT_REF)
    B_q = ORACLE.quantize(ol.Q8_1, rng.standard_normal((N, K), dtype=np.float32), ol.QUANT_AVX)
    c, packed = stationary(A_q, B_q, M, N, K)
    assert packed > 0
    rows = np.arange(M) if M <= 512 else np.unique(np.r_[np.arange(0, M, 16), [1, 255, 256, M - 1]])
    err = check(c, A_q, B_q, M, N, K, rows)
    print(f"q5_1 fp6 {M}x{N}x{K}: max rel err {err:.2e}")
    assert err < TOL


POS_SHAPES = [(300, 40, 96), (257, 64, 1024), (4096, 512, 1024)]


@pytest.mark.parametrize("shape", POS_SHAPES, ids=[f"{m}x{n}x{k}" for m, n, k in POS_SHAPES])
def test_q5_1_fp6_positive_activations(shape, monkeypatch):
    """the shift's affine term uses the activation block's rounded fp16 s = d_b sum q_b, so
    sum_b 16 d_a s_b differs from the reference's 16 d_a d_b sum q_b by 16 d_a (s_b - d_b sum q_b) per
    block.  Activations that never cancel (all positive: s_b large) and centred weights (|w| << 16 d,
    small sum |a b|) make that margin largest, most at small K.  Still within the bar."""
    M, N, K = shape
    if M * N < 4096 * 512:
        monkeypatch.setenv("LAMM_GEMM_PATH", "fp6")
    assert la.gemm_engine(T, M, N, K, 1, stationary=True) == "fp6"
    rng = np.random.default_rng(M * 7 + K)
    a = rng.standard_normal((M, K), dtype=np.float32) * 0.1   # centred: m ~ -16 d
    b = rng.random((N, K), dtype=np.float32) + 0.5            # all positive, no cancellation
    A_q = ORACLE.quantize(T, a, ol.QUANT_REF)
    B_q = ORACLE.quantize(ol.Q8_1, b, ol.QUANT_AVX)
    c, packed = stationary(A_q, B_q, M, N, K)
    assert packed > 0
    rows = np.arange(M) if M <= 512 else np.unique(np.r_[np.arange(0, M, 16), [1, 255, 256, M - 1]])
    err = check(c, A_q, B_q, M, N, K, rows)
    print(f"q5_1 fp6 positive activations {M}x{N}x{K}: max rel err {err:.2e}")
    assert err < TOL


def test_q5_1_per_call_stays_off_fp6(monkeypatch):
    """Without prepared weights q5_1 never reaches the fp6 engine (no range check per call): dq16 by
    default, the exact i8 engine when fp6 is forced."""
    assert la.gemm_engine(T, 4096, 512, 4096) == "dq16"
    monkeypatch.setenv("LAMM_GEMM_PATH", "fp6")
    assert la.gemm_engine(T, 4096, 512, 4096) == "i8"
    M, N, K = 257, 129, 4096 + 64
    rng = np.random.default_rng(4)
    A_q = ORACLE.quantize(T, rng.standard_normal((M, K), dtype=np.float32), ol.QUANT_REF)
    B_q = ORACLE.quantize(ol.Q8_1, rng.standard_normal((N, K), dtype=np.float32), ol.QUANT_AVX)
    kb = K // 32
    lda = pitch_blocks(T, kb)
    A = dev_bytes(pitched_A(T, A_q, M, kb, lda))
    C = torch.full((N * M,), float("nan"), dtype=torch.float32, device="cuda")
    la.mul_mat_torch(T, A, dev_bytes(B_q), C, M, N, K, lda=lda)
    torch.cuda.synchronize()
    assert check(C.cpu().numpy().reshape(N, M), A_q, B_q, M, N, K, np.arange(M)) < TOL


def test_q5_1_large_block_scale_falls_back():
    """A weight tensor with one block scale past 2047 (a block spanning -65000 .. 65000: d = 4193,
    m still inside f16): no packed form is kept and the call runs, finite and within the bar, on
    the range-guarded dq16 engine."""
    M, N, K = 4096, 512, 1024
    rng = np.random.default_rng(8)
    a = rng.standard_normal((M, K), dtype=np.float32)
    a[100, 32:64] = np.linspace(-65000.0, 65000.0, 32, dtype=np.float32)
    A_q = ORACLE.quantize(T, a, ol.QUANT_REF)
    B_q = ORACLE.quantize(ol.Q8_1, rng.standard_normal((N, K), dtype=np.float32), ol.QUANT_AVX)
    c, packed = stationary(A_q, B_q, M, N, K)
    assert packed == 0
    rows = np.unique(np.r_[np.arange(0, M, 32), [99, 100, 101]])
    assert check(c, A_q, B_q, M, N, K, rows) < TOL
