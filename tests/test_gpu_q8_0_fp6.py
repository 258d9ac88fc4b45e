"""q8_0 prefill on the EXACT block-scaled fp6 engine (round 6; lamm_gemm_fp6.hip
F6<kQ8_0>): the weight's quants q in [-127, 127] do not fit e2m3, so the weight prep splits them like the
activations, q = 16 h + l, into a hi and a lo code plane, and every unit's block dot is two chained scale
MFMAs (the hi one with its weight scale x16) -- S = sum q b exactly, then d_a d_b S as the reference's
lamm q8_0 kernel computes it (src/lamm_kernel_q8_0.hpp:50-117, the scalar restatement: the oracle).  Only
weight-stationary calls on the 128 x 64 K-group plan take it (config 4's shape; Llama prefill at N = 512);
everything else stays on the range-guarded dq16 engine."""
import numpy as np
import pytest

import oracle_lib as ol

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
import lamm_amd as la  # noqa: E402
from conftest import rel_err  # noqa: E402
from test_gpu_parity import TOL, absdot, dev_bytes, pitch_blocks, pitched_A  # noqa: E402

ORACLE = ol.Oracle()
T = ol.Q8_0


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
    assert np.isnan(c[N * M:]).all()   # nothing past C
    return c[:N * M].reshape(N, M), packed


def check(c, A_q, B_q, M, N, K, rows):
    arow = (K // 32) * la.type_size(T)
    A_s = np.ascontiguousarray(A_q).reshape(M, arow)[rows].reshape(-1)
    ref = ORACLE.mul_mat(T, len(rows), N, K, A_s, B_q)
    assert np.isfinite(c).all()
    return rel_err(c[:, rows], ref, absdot(T, A_s, B_q, len(rows), N, K)).max(), ref


SHAPES = [(4096, 512, 4096), (4096, 512, 1024), (11008, 512, 4096), (4096, 512, 11008)]


@pytest.mark.parametrize("shape", SHAPES, ids=[f"{m}x{n}x{k}" for m, n, k in SHAPES])
def test_q8_0_fp6_stationary_vs_oracle(shape):
    M, N, K = shape
    assert la.gemm_engine(T, M, N, K, 1, stationary=True) == "fp6"
    assert la.gemm_engine(T, M, N, K) == "dq16"      # the per-call form keeps dq16
    rng = np.random.default_rng(M + N + K)
    A_q = ORACLE.quantize(T, rng.standard_normal((M, K), dtype=np.float32))
    B_q = ORACLE.quantize(T, rng.standard_normal((N, K), dtype=np.float32), ol.QUANT_AVX)
    c, packed = stationary(A_q, B_q, M, N, K)
    assert packed >= M * (K // 32) * 64   # two 32-byte code planes per row and block
    rows = np.unique(np.r_[np.arange(0, M, 16), [1, 127, 128, M - 1]])
    err, _ = check(c, A_q, B_q, M, N, K, rows)
    print(f"q8_0 fp6 {M}x{N}x{K}: max rel err {err:.2e}")
    assert err < TOL


def test_q8_0_fp6_extreme_quants_exact():
    """Quants at both ends of int8 (the raw bytes +-127 and -128, every h / l combination) and
    integer-valued scales: the block dots are then exact integers on both sides, and the fp32 sums of
    d_a d_b S are exact too -- the GPU's C must equal the oracle's bit for bit."""
    M, N, K = 4096, 512, 1024
    rng = np.random.default_rng(88)
    kb = K // 32

    def blocks(rows, qs_choice):
        out = np.zeros((rows, kb, 34), np.uint8)
        out[:, :, 0:2] = np.frombuffer(np.float16(1.0).tobytes(), np.uint8)   # d = 1
        out[:, :, 2:] = rng.choice(qs_choice, size=(rows, kb, 32)).astype(np.int8).view(np.uint8)
        return out.reshape(-1)
    A_q = blocks(M, np.array([-128, -127, -1, 0, 1, 15, 16, 17, 127], np.int16))
    B_q = blocks(N, np.array([-127, -64, 0, 3, 64, 127], np.int16))
    c, _ = stationary(A_q, B_q, M, N, K)
    rows = np.arange(0, M, 8)
    err, ref = check(c, A_q, B_q, M, N, K, rows)
    assert np.array_equal(c[:, rows], ref), err


def test_q8_0_fp6_value_range():
    """Weights up to |w| = 300 and activations up to 1e5 (the bound the dq16 engine needs its range
    guard for): the exact engine has no f16 operands to overflow -- finite and within the bar."""
    M, N, K = 4096, 512, 1024
    rng = np.random.default_rng(5)
    a = rng.standard_normal((M, K), dtype=np.float32)
    a *= 300 / np.abs(a).max()
    b = rng.standard_normal((N, K), dtype=np.float32)
    b[: N // 2] *= 1e5 / np.abs(b).max()
    A_q = ORACLE.quantize(T, a)
    B_q = ORACLE.quantize(T, b, ol.QUANT_AVX)
    c, _ = stationary(A_q, B_q, M, N, K)
    rows = np.random.default_rng(0).choice(M, 256, replace=False)
    err, _ = check(c, A_q, B_q, M, N, K, rows)
    assert err < TOL


RAGGED = [(4000, 500, 4160), (4032, 456, 4128)]


@pytest.mark.parametrize("shape", RAGGED, ids=[f"{m}x{n}x{k}" for m, n, k in RAGGED])
def test_q8_0_fp6_ragged_vs_oracle(shape):
    """Shapes off every tile edge on the same exact engine: rows past the last 128-row tile, columns
    past the last 64-column tile and an odd number of blocks (a K-step of one block at the end, the
    two weight code planes' last chunk half empty) -- every row the oracle checks, nothing written
    past C."""
    M, N, K = shape
    assert la.gemm_engine(T, M, N, K, 1, stationary=True) == "fp6"
    rng = np.random.default_rng(M * 7 + N + K)
    A_q = ORACLE.quantize(T, rng.standard_normal((M, K), dtype=np.float32))
    B_q = ORACLE.quantize(T, rng.standard_normal((N, K), dtype=np.float32), ol.QUANT_AVX)
    c, _ = stationary(A_q, B_q, M, N, K)
    rows = np.unique(np.r_[np.arange(0, M, 7), np.arange(M - 40, M)])
    err, _ = check(c, A_q, B_q, M, N, K, rows)
    print(f"q8_0 fp6 ragged {M}x{N}x{K}: max rel err {err:.2e}")
    assert err < TOL
