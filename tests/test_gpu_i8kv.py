"""The int8 K-group engine (lamm_gemm_i8kv.hip, LAMM_I8KV=1): prepared q4_0 / q5_0 / q8_0 weights on the
128 x 64 K-group plan with the block dots on v_mfma_i32_32x32x32_i8 and ggml's q8_0 activation rows read
as they are stored (no activation prep launch).  Its S is the same exact integer the fp6 engine
computes, converted, then the same P-MFMA and FMA in the same order: C must equal the fp6 engine's bit
for bit, and the oracle within the bar (src/lamm_kernel_q4_0.hpp:59-128 and siblings)."""
import numpy as np
import pytest

import oracle_lib as ol

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
import lamm_amd as la  # noqa: E402
from conftest import rel_err  # noqa: E402
from test_gpu_parity import TOL, absdot, dev_bytes, pitch_blocks, pitched_A  # noqa: E402

ORACLE = ol.Oracle()
TYPES = [ol.Q4_0, ol.Q5_0, ol.Q8_0]
# config 3 / config 4; ragged M, N and an odd block count (row pitch 2 mod 4 bytes); a pitch of one
# block past the row (2 mod 4 again, the blocks' byte shifts alternating by row)
SHAPES = [(4096, 512, 4096, 0), (4000, 500, 4160, 0), (2048, 300, 3104, 0), (4096, 512, 1024, 1)]


def run(t, A_q, B_q, M, N, K, i8, ldb_pad, monkeypatch):
    monkeypatch.setenv("LAMM_I8KV", "1" if i8 else "0")
    la.reload_env()
    kb = K // 32
    lda = pitch_blocks(t, kb)
    A = dev_bytes(pitched_A(t, A_q, M, kb, lda))
    rowb = kb * 34
    ldb = kb + ldb_pad   # in blocks
    Bp = np.zeros((N, ldb * 34), np.uint8)
    Bp[:, :rowb] = B_q.reshape(N, rowb)
    B = dev_bytes(Bp.reshape(-1))
    C = torch.full((N * M + 16,), float("nan"), dtype=torch.float32, device="cuda")
    W = la.Weights(t, A, M, K, lda=lda)
    W.matmul_torch(B, C, N, ldb=ldb)
    torch.cuda.synchronize()
    W.close()
    c = C.cpu().numpy()
    assert np.isnan(c[N * M:]).all()
    return c[:N * M].reshape(N, M)


@pytest.mark.parametrize("t", TYPES, ids=[ol.NAMES[t] for t in TYPES])
@pytest.mark.parametrize("shape", SHAPES, ids=[f"{m}x{n}x{k}+{p}" for m, n, k, p in SHAPES])
def test_i8kv_bit_identical_to_fp6_and_oracle(t, shape, monkeypatch):
    M, N, K, pad = shape
    rng = np.random.default_rng(M * 3 + N + K + t)
    A_q = ORACLE.quantize(t, rng.standard_normal((M, K), dtype=np.float32))
    B_q = ORACLE.quantize(ol.Q8_0, rng.standard_normal((N, K), dtype=np.float32), ol.QUANT_AVX)
    try:
        c_fp6 = run(t, A_q, B_q, M, N, K, False, pad, monkeypatch)
        c_i8 = run(t, A_q, B_q, M, N, K, True, pad, monkeypatch)
    finally:
        monkeypatch.delenv("LAMM_I8KV", raising=False)
        la.reload_env()
    assert np.array_equal(c_i8.view(np.uint32), c_fp6.view(np.uint32)), f"{(c_i8 != c_fp6).sum()} differ"
    rows = np.unique(np.r_[np.arange(0, M, 97), [M - 1]])
    arow = (K // 32) * la.type_size(t)
    A_s = np.ascontiguousarray(A_q).reshape(M, arow)[rows].reshape(-1)
    ref = ORACLE.mul_mat(t, len(rows), N, K, A_s, B_q)
    assert rel_err(c_i8[:, rows], ref, absdot(t, A_s, B_q, len(rows), N, K)).max() < TOL
