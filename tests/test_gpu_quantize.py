"""GPU activation quantizers bit-exact against the reference's
own bytes: B_ref = from_float_reference, B_avx = AVX2 from_float (golden vectors)."""
import numpy as np
import pytest

from conftest import fixture_paths, load_fixture, load_inputs
import oracle_lib as ol

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
import lamm_amd as la  # noqa: E402

FIXTURES = [p for p in fixture_paths() if not p.rsplit("/", 1)[-1].startswith("f32")]


def gpu_quant(vt, x, flavour):
    N, K = x.shape
    xd = torch.from_numpy(np.ascontiguousarray(x)).cuda()
    nbytes = la.row_bytes(vt, K) * N
    y = torch.zeros(nbytes + 16, dtype=torch.uint8, device="cuda")
    la.quantize_torch(vt, xd, y, flavour=flavour)
    torch.cuda.synchronize()
    return y.cpu().numpy()[:nbytes]


@pytest.mark.parametrize("path", FIXTURES, ids=[p.rsplit("/", 1)[-1][:-4] for p in FIXTURES])
def test_quantizer_matches_reference_bytes(path):
    z = load_fixture(path)
    vt, M, N, K = int(z["vdt"]), int(z["M"]), int(z["N"]), int(z["K"])
    _, b = load_inputs(M, N, K)
    assert np.array_equal(gpu_quant(vt, b, 0), z["B_ref"])
    if vt != ol.Q8_K:
        assert np.array_equal(gpu_quant(vt, b, 1), z["B_avx"])


@pytest.mark.parametrize("vt", [ol.Q8_0, ol.Q8_1, ol.Q8_K], ids=["q8_0", "q8_1", "q8_k"])
def test_quantizer_edge_values(vt):
    o = ol.Oracle()
    K = 1024
    rng = np.random.default_rng(3)
    x = np.stack([
        rng.standard_normal(K).astype(np.float32) * 1e-3,
        np.zeros(K, np.float32),                          # amax == 0 branch
        np.repeat(np.float32([0.5, -0.5, 1.5, -2.5]), K // 4),  # exact .5 ties
        (rng.standard_normal(K) * 1e4).astype(np.float32),
    ])
    flavours = [0] if vt == ol.Q8_K else [0, 1]
    for f in flavours:
        assert np.array_equal(gpu_quant(vt, x, f), o.quantize(vt, x, f)), f"flavour {f}"


# Weight quantizers (ggml_quantize_chunk, LC/ggml.c:20413, no importance matrix): the GPU
# bytes must equal the reference's own quantized A (A_q, made by the real reference from
# the same f32 inputs) for every weight type, k-quants included.
A_FIXTURES = [p for p in fixture_paths() if not p.rsplit("/", 1)[-1].startswith("f32")]


@pytest.mark.parametrize("path", A_FIXTURES, ids=[p.rsplit("/", 1)[-1][:-4] for p in A_FIXTURES])
def test_weight_quantizer_matches_reference_bytes(path):
    z = load_fixture(path)
    t, M, N, K = int(z["type"]), int(z["M"]), int(z["N"]), int(z["K"])
    a, _ = load_inputs(M, N, K)
    got = gpu_quant(t, a, 0)
    want = z["A_q"]
    bad = np.flatnonzero(got != want)
    assert bad.size == 0, f"{bad.size} bytes differ, first at {bad[:8]} (block {bad[0] // la.type_size(t)})"


@pytest.mark.parametrize("t", [ol.Q4_0, ol.Q4_1, ol.Q5_0, ol.Q5_1, ol.Q8_0, ol.Q2_K],
                         ids=["q4_0", "q4_1", "q5_0", "q5_1", "q8_0", "q2_k"])
def test_weight_quantizer_edge_values(t):
    """Zero rows, constant rows (the la-benchmark-matmult inputs), exact ties, tiny and
    huge magnitudes, mixed signs: GPU bytes == the oracle's restated reference quantizer."""
    o = ol.Oracle()
    K = 1024
    rng = np.random.default_rng(11)
    x = np.stack([
        np.zeros(K, np.float32),
        np.full(K, 1.0, np.float32), np.full(K, 1.5, np.float32), np.full(K, -2.0, np.float32),
        np.repeat(np.float32([0.5, -0.5, 1.5, -2.5, 3.5, -7.5, 8.0, -8.0]), K // 8),
        rng.standard_normal(K).astype(np.float32) * 1e-4,
        (rng.standard_normal(K) * 1e3).astype(np.float32),
        np.abs(rng.standard_normal(K)).astype(np.float32) + 1.0,
        rng.uniform(1, 2, K).astype(np.float32),
    ])
    assert np.array_equal(gpu_quant(t, x, 0), o.quantize(t, x, 0))


def test_weight_quantizer_kquants_constant_rows():
    """k-quants on the la-benchmark-matmult constant inputs (A = 1.0 / 1.5): dequantised
    values reproduce the constant (no oracle quantizer for q4_K/q5_K/q6_K; checked by
    dequantising with the oracle's pinned dequantizer)."""
    o = ol.Oracle()
    K = 512
    for t in ol.KQ_TYPES:
        for c in (1.0, 1.5, -2.0, 0.0):
            x = np.full((2, K), c, np.float32)
            q = gpu_quant(t, x, 0)
            d = o.dequantize(t, q, 2, K)
            assert np.allclose(d, c, rtol=2e-3, atol=0), (ol.NAMES[t], c, d[0, :4])


@pytest.mark.parametrize("vt", [ol.Q8_0, ol.Q8_1], ids=["q8_0", "q8_1"])
def test_quantizer_id_inf_blocks(vt):
    """0 < amax < ~3.7e-37 makes the AVX2 flavour's id = 127 / amax infinite: x * id is inf (NaN
    for zeros) and _mm256_cvtps_epi32 gives INT_MIN, -128 after the packs (v_cvt_i32_f32 would
    saturate to INT_MAX instead) -- the device quantizer emulates the x86 conversion."""
    o = ol.Oracle()
    K = 1024
    rng = np.random.default_rng(5)
    x = (rng.standard_normal((3, K)) * 1e-38).astype(np.float32)
    x[1, 32:64] = 0.0
    x[1, 40] = 1e-39
    x[2, ::3] = 0.0
    assert np.array_equal(gpu_quant(vt, x, 1), o.quantize(vt, x, 1))
