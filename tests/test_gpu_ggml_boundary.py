"""The drop-in boundary on the GPU: lamm_can_mul_mat / lamm_mul_mat driven exactly as
ggml_compute_forward_mul_mat drives the reference plug-in (tests/ggml_emu.py)."""
import numpy as np
import pytest

from conftest import rel_err
import oracle_lib as ol

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
import lamm_amd as la  # noqa: E402
import ggml_emu  # noqa: E402

ORACLE = ol.Oracle()


def make_node(t, M, N, K, ne2=(1, 1), ne3=(1, 1), seed=0, transpose_free=True):
    """src0 [K, M, ne02, ne03] of type t, src1 F32 [K, N, ne12, ne13]."""
    rng = np.random.default_rng(seed)
    n0 = ne2[0] * ne3[0]
    n1 = ne2[1] * ne3[1]
    a = rng.standard_normal((n0 * M, K), dtype=np.float32)
    b = rng.standard_normal((n1 * N, K), dtype=np.float32)
    A_q = ORACLE.quantize(t, a)
    src0 = ggml_emu.Tensor(t, [K, M, ne2[0], ne3[0]], data=A_q)
    src1 = ggml_emu.Tensor(ol.F32, [K, N, ne2[1], ne3[1]], data=b)
    return src0, src1, A_q, b


def expected(t, A_q, b, M, N, K, ne2, ne3):
    """ggml semantics incl. broadcast r2 = ne12/ne02, r3 = ne13/ne03."""
    vt = la.vec_dot_type(t)
    fl = ol.QUANT_AVX if vt in (ol.Q8_0, ol.Q8_1) else ol.QUANT_REF
    arow, brow = ORACLE.row_bytes(t, K), ORACLE.row_bytes(vt, K)
    B_q = ORACLE.quantize(vt, b, fl)
    r2, r3 = ne2[1] // ne2[0], ne3[1] // ne3[0]
    out = np.zeros((ne3[1], ne2[1], N, M), np.float32)
    for i13 in range(ne3[1]):
        for i12 in range(ne2[1]):
            a_slice = (i13 // r3) * ne2[0] + i12 // r2
            b_slice = i13 * ne2[1] + i12
            A = A_q[a_slice * M * arow:(a_slice + 1) * M * arow]
            B = B_q[b_slice * N * brow:(b_slice + 1) * N * brow]
            out[i13, i12] = ORACLE.mul_mat(t, M, N, K, A, B)
    return out


@pytest.mark.parametrize("t", ol.A_TYPES, ids=[ol.NAMES[t] for t in ol.A_TYPES])
def test_boundary_matches_oracle(t, monkeypatch):
    """Both INIT modes: src1 quantized on the GPU (default) and by ggml's CPU INIT
    (LAMM_HIP_GPU_QUANT=0).  The GPU quantizer is bit-exact with the AVX2 from_float the
    CPU path uses, so the two outputs must be identical bit for bit."""
    M, N, K = 67, 9, 512
    outs = []
    for mode in ("1", "0"):
        monkeypatch.setenv("LAMM_HIP_GPU_QUANT", mode)
        src0, src1, A_q, b = make_node(t, M, N, K, seed=t)
        dst = ggml_emu.mul_mat_node(src0, src1)
        assert ggml_emu.compute(dst, nth=3) is True
        got = dst.buf.view(np.float32).reshape(N, M)
        want = expected(t, A_q, b, M, N, K, (1, 1), (1, 1))[0, 0]
        assert rel_err(got, want, np.abs(want) + 1.0).max() < 1e-3
        outs.append(got.copy())
    if t not in (ol.F32,):
        np.testing.assert_array_equal(outs[0], outs[1])
    assert la.get_opt_level() == 3


def test_boundary_batch_broadcast():
    """ne02=2 weights broadcast over ne12=4 activations (r2=2), ne13=2 over ne03=1."""
    t, M, N, K = ol.Q4_0, 32, 5, 256
    ne2, ne3 = (2, 4), (1, 2)
    src0, src1, A_q, b = make_node(t, M, N, K, ne2, ne3, seed=11)
    dst = ggml_emu.mul_mat_node(src0, src1)
    assert ggml_emu.compute(dst, nth=4)
    got = dst.buf.view(np.float32).reshape(ne3[1], ne2[1], N, M)
    want = expected(t, A_q, b, M, N, K, ne2, ne3)
    assert rel_err(got, want, np.abs(want) + 1.0).max() < 1e-3


def test_weight_cache_reuse_and_invalidation():
    t, M, N, K = ol.Q8_0, 64, 2, 1024
    la.cache_clear()
    src0, src1, A_q, b = make_node(t, M, N, K, seed=5)
    dst = ggml_emu.mul_mat_node(src0, src1)
    ggml_emu.compute(dst)
    first = dst.buf.view(np.float32).copy()
    used = la.cache_bytes()
    assert used > 0
    ggml_emu.compute(dst)                       # same weights: served from the cache
    assert la.cache_bytes() == used
    assert np.array_equal(first, dst.buf.view(np.float32))
    # overwrite the host weights in place (same pointer): fingerprint must catch it
    new_q = ORACLE.quantize(t, np.random.default_rng(6).standard_normal((M, K), dtype=np.float32))
    src0.buf[:] = new_q
    ggml_emu.compute(dst)
    want = expected(t, new_q, b, M, N, K, (1, 1), (1, 1))[0, 0]
    got = dst.buf.view(np.float32).reshape(N, M)
    assert rel_err(got, want, np.abs(want) + 1.0).max() < 1e-3
    la.cache_clear()
    assert la.cache_bytes() == 0


def test_non_compute_phases_and_unsupported(monkeypatch):
    t, M, N, K = ol.Q4_0, 16, 1, 256
    src0, src1, _, _ = make_node(t, M, N, K)
    dst = ggml_emu.mul_mat_node(src0, src1)
    p = la.GgmlComputeParams()
    p.ith, p.nth = 0, 1
    p.type = la.TASK_FINALIZE
    assert not la.can_mul_mat(p, dst.t)
    p.type = la.TASK_INIT        # claimed only when src1 is quantized on the GPU
    assert not la.can_mul_mat(p, dst.t)          # default: N = 1 stays on ggml's CPU INIT
    monkeypatch.setenv("LAMM_HIP_GPU_QUANT", "1")
    assert la.can_mul_mat(p, dst.t)
    monkeypatch.setenv("LAMM_HIP_GPU_QUANT", "0")
    assert not la.can_mul_mat(p, dst.t)
    monkeypatch.delenv("LAMM_HIP_GPU_QUANT")
    src0b, src1b, _, _ = make_node(t, M, 8, K)   # from 8 activation rows: GPU quantizer
    dstb = ggml_emu.mul_mat_node(src0b, src1b)
    assert la.can_mul_mat(p, dstb.t)
    p.type = la.TASK_COMPUTE
    assert la.can_mul_mat(p, dst.t)
    src0.t.type = 1  # F16 src0 (KV cache matmuls): not on the lamm path
    assert not la.can_mul_mat(p, dst.t)
