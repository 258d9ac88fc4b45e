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
