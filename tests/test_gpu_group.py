"""lamm_hip_matmul_group (csrc/lamm_hip.cpp; ref_gemv_group_kernel in csrc/lamm_ref.hip,
gemv_flat_group_kernel in csrc/lamm_gemv_rpw.hip): several weights times one activation column -- wq /
wk / wv, ffn gate / up (LC/llama.cpp:5738-5752) -- must give every C[i] the bits of its own
lamm_hip_matmul_ex call, in one launch for reference-order calls and for fast-order K = 4096 weights of
>= 2048 rows, and through the per-weight fallback for anything else; the reference-order results are
the oracle's AVX2-order bits, the fast-order ones within the north star's 1e-3."""
import numpy as np
import pytest

import oracle_lib as ol

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
import lamm_amd as la  # noqa: E402
from test_gpu_parity import dev_bytes, pitch_blocks, pitched_A  # noqa: E402

ORACLE = ol.Oracle()
REF_TYPES = [ol.Q4_0, ol.Q4_1, ol.Q5_0, ol.Q5_1]


def bits(x):
    return np.ascontiguousarray(x, dtype=np.float32).view(np.uint32)


def weights(t, Ms, K, seed):
    rng = np.random.default_rng(seed)
    kb = K // 32
    lda = pitch_blocks(t, kb)
    qs, keep, mats = [], [], []
    for M in Ms:
        A_q = ORACLE.quantize(t, rng.standard_normal((M, K), dtype=np.float32), ol.QUANT_REF)
        A = dev_bytes(pitched_A(t, A_q, M, kb, lda))
        qs.append(A_q)
        keep.append(A)
        mats.append(la.Matrix(A.data_ptr(), t, M, kb, lda))
    return qs, keep, mats


def activation(t, K, f32_rows, seed):
    x = np.random.default_rng(seed).standard_normal((1, K)).astype(np.float32)
    kb = K // 32
    Bq = ORACLE.quantize(la.vec_dot_type(t), x, ol.QUANT_AVX)
    if f32_rows:
        B = torch.from_numpy(x.reshape(-1)).to("cuda")
        return B, la.Matrix(B.data_ptr(), la.F32, K, 1, K), Bq
    B = dev_bytes(Bq)
    return B, la.Matrix(B.data_ptr(), la.vec_dot_type(t), kb, 1, kb), Bq


def outputs(Ms):
    Cs = [torch.full((M + 16,), float("nan"), dtype=torch.float32, device="cuda") for M in Ms]
    return Cs, [la.Matrix(C.data_ptr(), la.F32, M, 1, M) for C, M in zip(Cs, Ms)]


def run(Ams, Bm, Ms, flags, group):
    stream = torch.cuda.current_stream().cuda_stream
    Cs, Cms = outputs(Ms)
    if group:
        la.matmul_group(Ams, Bm, Cms, flags, stream)
    else:
        for Am, Cm in zip(Ams, Cms):
            la.matmul_ex(Am, Bm, Cm, None, flags, stream)
    torch.cuda.synchronize()
    out = [C.cpu().numpy() for C in Cs]
    for o, M in zip(out, Ms):
        assert np.isnan(o[M:]).all()   # nothing past the rows
    return [o[:M] for o, M in zip(out, Ms)]


@pytest.mark.parametrize("t", REF_TYPES, ids=[ol.NAMES[t] for t in REF_TYPES])
@pytest.mark.parametrize("Ms,K", [((4096, 4096, 4096), 4096), ((11008, 11008), 4096), ((4096, 1024, 67, 13), 4096),
                                  ((5120, 5120, 5120), 5120), ((4096, 2048), 8192)],
                         ids=["qkv", "gate_up", "ragged4", "qkv_k5120", "k8192"])
@pytest.mark.parametrize("f32_rows", [False, True], ids=["q8_rows", "f32_rows"])
def test_group_reference_order_bitwise(t, Ms, K, f32_rows):
    """K = 5120 / 8192 (13B / 70B hidden sizes): the single reference-order launch switches
    to 128-block chunks beyond K = 4096 while the group kernel keeps 64-block chunks -- the chained
    lane order must not depend on the chunking."""
    qs, keep, Ams = weights(t, Ms, K, seed=len(Ms) * 100 + t)
    B, Bm, Bq = activation(t, K, f32_rows, seed=t + 3)
    one = run(Ams, Bm, Ms, la.ORDER_REFERENCE, False)
    grp = run(Ams, Bm, Ms, la.ORDER_REFERENCE, True)
    for i, (a, b) in enumerate(zip(one, grp)):
        assert np.array_equal(bits(a), bits(b)), f"weight {i}"
    # and the oracle's reference (AVX2 lane) order, for the shortest weight
    i = int(np.argmin(Ms))
    want = ORACLE.mul_mat_avx(t, Ms[i], 1, K, qs[i], Bq)[0]
    assert np.array_equal(bits(grp[i]), bits(want))


FAST_TYPES = [ol.Q4_0, ol.Q4_1, ol.Q5_0, ol.Q5_1, ol.Q8_0]


@pytest.mark.parametrize("t", FAST_TYPES, ids=[ol.NAMES[t] for t in FAST_TYPES])
@pytest.mark.parametrize("Ms", [(4096, 4096, 4096), (11008, 11008), (4096, 2048, 3000, 11008)],
                         ids=["qkv", "gate_up", "ragged4"])
@pytest.mark.parametrize("f32_rows", [False, True], ids=["q8_rows", "f32_rows"])
def test_group_fast_order_bitwise(t, Ms, f32_rows):
    """The fast order (the ggml boundary's default since round 6): one gemv_flat_group_kernel launch,
    every weight's C the bits of its single call (gemv_flat1_kernel), and within 1e-3 of the oracle."""
    K = 4096
    qs, keep, Ams = weights(t, Ms, K, seed=len(Ms) * 10 + t)
    B, Bm, Bq = activation(t, K, f32_rows, seed=t + 5)
    one = run(Ams, Bm, Ms, 0, False)
    grp = run(Ams, Bm, Ms, 0, True)
    for i, (a, b) in enumerate(zip(one, grp)):
        assert np.array_equal(bits(a), bits(b)), f"weight {i}"
    for i in range(len(Ms)):
        want = ORACLE.mul_mat(t, Ms[i], 1, K, qs[i], Bq)[0]
        Ad = ORACLE.dequantize(t, qs[i], Ms[i], K).astype(np.float64)
        absdot = np.abs(Ad) @ np.abs(ORACLE.dequantize(la.vec_dot_type(t), Bq, 1, K).astype(np.float64))[0]
        assert (np.abs(grp[i] - want) / np.maximum(absdot, 1e-30)).max() < 1e-3


def test_group_fallbacks_and_errors():
    """Fast order, two columns, mixed types and K: one call per weight, the same bits; n outside
    1..GROUP_MAX is an error."""
    K = 4096
    stream = torch.cuda.current_stream().cuda_stream
    qs, keep, Ams = weights(ol.Q4_0, (4096, 512), K, seed=1)
    B, Bm, _ = activation(ol.Q4_0, K, False, seed=2)
    assert all(np.array_equal(bits(a), bits(b))
               for a, b in zip(run(Ams, Bm, (4096, 512), 0, False), run(Ams, Bm, (4096, 512), 0, True)))
    # mixed types: q4_0 and q5_0 share q8_0 activations
    qs2, keep2, Ams2 = weights(ol.Q5_0, (256,), K, seed=4)
    mix = [Ams[0], Ams2[0]]
    Ms = (4096, 256)
    assert all(np.array_equal(bits(a), bits(b))
               for a, b in zip(run(mix, Bm, Ms, la.ORDER_REFERENCE, False), run(mix, Bm, Ms, la.ORDER_REFERENCE, True)))
    # a single weight
    assert np.array_equal(bits(run(Ams[:1], Bm, (4096,), la.ORDER_REFERENCE, True)[0]),
                          bits(run(Ams[:1], Bm, (4096,), la.ORDER_REFERENCE, False)[0]))
    Cs, Cms = outputs((4096,) * 5)
    with pytest.raises(la.LammError):
        la.matmul_group([Ams[0]] * 5, Bm, Cms, la.ORDER_REFERENCE, stream)
    with pytest.raises(la.LammError):
        la.matmul_group([], Bm, [], la.ORDER_REFERENCE, stream)
