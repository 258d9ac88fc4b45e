"""The super-block GEMM (lamm_gemm_kq.hip, q2_K / q4_K / q5_K / q6_K x q8_K) with its B chunk DMA'd straight
from ggml's q8_K rows (round 6, the default) against the prep_b_kq launch it replaces (LAMM_KQ_RAWB=0):
the same LDS image and arithmetic, so C must be identical bit for bit -- on ragged M / N, the split-K plan
(few tiles), a row pitch past the row, batch slices broadcasting one weight slice, and weight-stationary
calls (config 4's q2_K shape)."""
import numpy as np
import pytest

import oracle_lib as ol

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
import lamm_amd as la  # noqa: E402
from test_gpu_parity import dev_bytes, pitch_blocks, pitched_A  # noqa: E402

ORACLE = ol.Oracle()
TYPES = [ol.Q2_K, ol.Q4_K, ol.Q5_K, ol.Q6_K]
SHAPES = [(4096, 512, 4096, 0), (300, 129, 2048, 1), (257, 40, 1024, 0), (64, 300, 256, 2), (4096, 32, 11008, 0)]


def blocks(t, M, K, rng):
    if t == ol.Q2_K:
        return ORACLE.quantize(t, rng.standard_normal((M, K), dtype=np.float32))
    return ol.random_kq_blocks(t, M, K, rng)


def run(t, A_q, B_q, M, N, K, pad, raw, stationary, monkeypatch):
    monkeypatch.setenv("LAMM_KQ_RAWB", "1" if raw else "0")
    la.reload_env()
    kb = K // 256
    lda = pitch_blocks(t, kb)
    A = dev_bytes(pitched_A(t, A_q, M, kb, lda))
    ldb = kb + pad   # q8_K blocks per B row (a pitch past the row: rows 292 * pad bytes apart more)
    Bp = np.zeros((N, ldb * 292), np.uint8)
    Bp[:, :kb * 292] = B_q.reshape(N, kb * 292)
    B = dev_bytes(Bp.reshape(-1))
    C = torch.full((N * M + 16,), float("nan"), dtype=torch.float32, device="cuda")
    if stationary:
        W = la.Weights(t, A, M, K, lda=lda)
        W.matmul_torch(B, C, N, ldb=ldb)
        torch.cuda.synchronize()
        W.close()
    else:
        la.mul_mat_torch(t, A, B, C, M, N, K, lda=lda, ldb=ldb)
        torch.cuda.synchronize()
    c = C.cpu().numpy()
    assert np.isnan(c[N * M:]).all()
    return c[:N * M].reshape(N, M)


@pytest.mark.parametrize("stationary", [False, True], ids=["per_call", "stationary"])
@pytest.mark.parametrize("t", TYPES, ids=[ol.NAMES[t] for t in TYPES])
@pytest.mark.parametrize("shape", SHAPES, ids=[f"{m}x{n}x{k}+{p}" for m, n, k, p in SHAPES])
def test_kq_raw_b_bit_identical(t, shape, stationary, monkeypatch):
    M, N, K, pad = shape
    rng = np.random.default_rng(M + 7 * N + K + t)
    A_q = blocks(t, M, K, rng)
    B_q = ORACLE.quantize(ol.Q8_K, rng.standard_normal((N, K), dtype=np.float32), ol.QUANT_REF)
    try:
        c0 = run(t, A_q, B_q, M, N, K, pad, False, stationary, monkeypatch)
        c1 = run(t, A_q, B_q, M, N, K, pad, True, stationary, monkeypatch)
    finally:
        monkeypatch.delenv("LAMM_KQ_RAWB", raising=False)
        la.reload_env()
    assert np.isfinite(c1).all()
    assert np.array_equal(c1.view(np.uint32), c0.view(np.uint32)), f"{(c1 != c0).sum()} of {c1.size} differ"
