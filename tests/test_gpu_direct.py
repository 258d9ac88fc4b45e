"""Direct dispatch (csrc/lamm_aql.cpp; lamm_hip_direct_begin / end): the one-kernel decode GEMVs
written as AQL packets into the library's own queue must compute the same bits as the same kernels
launched through HIP -- the flat config-2 GEMV (fast order) and the reference-order GEMV (F32 and
q8 activation rows) -- across the queue's ring of packets and kernarg slots, and a launch the
queue does not take (another kernel) must still run, through HIP."""
import numpy as np
import pytest

import oracle_lib as ol

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
import lamm_amd as la  # noqa: E402
from test_gpu_parity import dev_bytes, pitch_blocks, pitched_A  # noqa: E402

ORACLE = ol.Oracle()
FAST_TYPES = [ol.Q4_0, ol.Q4_1, ol.Q5_0, ol.Q5_1, ol.Q8_0]
REF_TYPES = [ol.Q4_0, ol.Q4_1, ol.Q5_0, ol.Q5_1]


def bits(x):
    return np.ascontiguousarray(x, dtype=np.float32).view(np.uint32)


def setup(t, M, K, f32_rows, seed):
    rng = np.random.default_rng(seed)
    A_q = ORACLE.quantize(t, rng.standard_normal((M, K), dtype=np.float32), ol.QUANT_REF)
    kb = K // 32
    lda = pitch_blocks(t, kb)
    A = dev_bytes(pitched_A(t, A_q, M, kb, lda))
    x = rng.standard_normal((1, K)).astype(np.float32)
    if f32_rows:
        B = torch.from_numpy(x.reshape(-1)).to("cuda")
        Bm = la.Matrix(B.data_ptr(), la.F32, K, 1, K)
    else:
        B = dev_bytes(ORACLE.quantize(la.vec_dot_type(t), x, ol.QUANT_AVX))
        Bm = la.Matrix(B.data_ptr(), la.vec_dot_type(t), kb, 1, kb)
    C = torch.full((M + 16,), float("nan"), dtype=torch.float32, device="cuda")
    Am = la.Matrix(A.data_ptr(), t, M, kb, lda)
    Cm = la.Matrix(C.data_ptr(), la.F32, M, 1, M)
    return (A, B, C), Am, Bm, Cm


def run_both(Am, Bm, Cm, C, M, flags):
    stream = torch.cuda.current_stream().cuda_stream
    C.fill_(float("nan"))
    la.matmul_ex(Am, Bm, Cm, None, flags, stream)
    torch.cuda.synchronize()
    via_hip = C.cpu().numpy()[:M].copy()
    C.fill_(float("nan"))
    torch.cuda.synchronize()
    with la.direct(torch.cuda.current_device()) as d:
        la.matmul_ex(Am, Bm, Cm, None, flags, stream)
    got = C.cpu().numpy()[:M].copy()
    return via_hip, got, d.launches


@pytest.mark.parametrize("t", FAST_TYPES, ids=[ol.NAMES[t] for t in FAST_TYPES])
@pytest.mark.parametrize("f32_rows", [False, True], ids=["q8_rows", "f32_rows"])
def test_direct_flat_gemv_bitwise(t, f32_rows):
    """Config 2's kernel (gemv_flat1_kernel: one column, K = 4096) on the direct queue."""
    M, K = 4096, 4096
    keep, Am, Bm, Cm = setup(t, M, K, f32_rows, seed=t + 11)
    via_hip, got, n = run_both(Am, Bm, Cm, keep[2], M, 0)
    assert n == (1 if t == ol.Q4_0 else n)   # q4_0: the flat kernel; the others as rpw_waves picks
    assert np.array_equal(bits(got), bits(via_hip))
    assert np.isfinite(got).all()


@pytest.mark.parametrize("t", REF_TYPES, ids=[ol.NAMES[t] for t in REF_TYPES])
@pytest.mark.parametrize("shape", [(4096, 4096), (67, 4096), (4096, 11008), (13, 4096 + 32 * 5)],
                         ids=["4096x4096", "67x4096", "4096x11008", "13x4256"])
@pytest.mark.parametrize("f32_rows", [False, True], ids=["q8_rows", "f32_rows"])
def test_direct_reference_gemv_bitwise(t, shape, f32_rows):
    """The boundary's decode kernel (ref_gemv_kernel, the reference's float order) on the direct
    queue: the same bits as through HIP, and as the oracle's AVX2 order."""
    M, K = shape
    keep, Am, Bm, Cm = setup(t, M, K, f32_rows, seed=M + K + t)
    via_hip, got, n = run_both(Am, Bm, Cm, keep[2], M, la.ORDER_REFERENCE)
    assert n == 1
    assert np.array_equal(bits(got), bits(via_hip))


def test_direct_ring_wraps_and_other_kernels_fall_back():
    """600 dispatches in one region (more than the 256-packet queue and the 512 kernarg slots),
    rotating over three weight copies: the last result of each copy matches its HIP launch; a
    two-column call (another kernel) inside the region goes through HIP and is counted as such."""
    M, K = 4096, 4096
    t = ol.Q4_0
    sets = [setup(t, M, K, False, seed=s) for s in range(3)]
    stream = torch.cuda.current_stream().cuda_stream
    want = []
    for keep, Am, Bm, Cm in sets:
        la.matmul_ex(Am, Bm, Cm, None, 0, stream)
        torch.cuda.synchronize()
        want.append(keep[2].cpu().numpy()[:M].copy())
        keep[2].fill_(float("nan"))
    torch.cuda.synchronize()
    with la.direct(torch.cuda.current_device()) as d:
        for i in range(600):
            _, Am, Bm, Cm = sets[i % 3]
            la.matmul_ex(Am, Bm, Cm, None, 0, stream)
    assert d.launches == 600
    for (keep, _, _, _), w in zip(sets, want):
        assert np.array_equal(bits(keep[2].cpu().numpy()[:M]), bits(w))
    # N = 3: not a direct-queue kernel -> HIP, inside an open region
    rng = np.random.default_rng(5)
    keep, Am, _, _ = sets[0]
    kb = K // 32
    x = rng.standard_normal((3, K)).astype(np.float32)
    B3 = dev_bytes(ORACLE.quantize(ol.Q8_0, x, ol.QUANT_AVX))
    C3 = torch.full((3 * M,), float("nan"), dtype=torch.float32, device="cuda")
    Bm3 = la.Matrix(B3.data_ptr(), ol.Q8_0, kb, 3, kb)
    Cm3 = la.Matrix(C3.data_ptr(), la.F32, M, 3, M)
    with la.direct(torch.cuda.current_device()) as d3:
        la.matmul_ex(Am, Bm3, Cm3, None, 0, stream)
    torch.cuda.synchronize()
    assert d3.launches == 0
    got = C3.cpu().numpy().reshape(3, M)
    C3.fill_(float("nan"))
    la.matmul_ex(Am, Bm3, Cm3, None, 0, stream)
    torch.cuda.synchronize()
    assert np.array_equal(bits(got), bits(C3.cpu().numpy().reshape(3, M)))


def test_direct_region_errors():
    dev = torch.cuda.current_device()
    with la.direct(dev):
        with pytest.raises(la.LammError):   # one region per thread
            with la.direct(dev):
                pass
    with pytest.raises(la.LammError):
        with la.direct(dev + 64):
            pass
