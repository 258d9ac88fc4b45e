"""The boundary's host activation quantizer (lamm_hip_quantize_host, lamm_host_quant.cpp) against
the oracle's AVX2 from_float restatement (LC/ggml-quants.c:1277-1330 / :1505-1575): byte for byte,
on the CPU (no device needed).  The prefill path (LAMM_HIP_POOL bit 1) uploads these bytes in
place of ggml's INIT output / the device quantizer's, so they must be identical."""
import ctypes
import os
import time

import numpy as np
import pytest

import lamm_amd as la
import oracle_lib as ol

ORACLE = ol.Oracle()
Q8 = [ol.Q8_0, ol.Q8_1]


def host_quant(t, x):
    x = np.ascontiguousarray(x, dtype=np.float32)
    rows, k = x.shape
    rb = ORACLE.row_bytes(t, k)
    out = np.zeros(rows * rb, dtype=np.uint8)
    for r in range(rows):
        rc = la.lib.lamm_hip_quantize_host(t, x[r].ctypes.data_as(ctypes.c_void_p),
                                           out[r * rb:].ctypes.data_as(ctypes.c_void_p), ctypes.c_int64(k))
        assert rc == 0
    return out


def cases(rng):
    k = 4096
    yield "normal", rng.standard_normal((16, k), dtype=np.float32)
    yield "wide_range", (rng.standard_normal((8, k)) * 10.0 ** rng.uniform(-6, 6, (8, k))).astype(np.float32)
    z = rng.standard_normal((4, k), dtype=np.float32)
    z[:, :32] = 0.0                                   # an all-zero block: d = 0, id = 0
    z[:, 64:96] = -0.0
    yield "zero_blocks", z
    # exact ties: amax = 127 makes id = 1, so x * id = x lands on .5 -> round half to even
    t = np.tile(np.array([127.0, -127.0, 2.5, -2.5, 3.5, -3.5, 0.5, -0.5, 1.5, -1.5, 126.5, -126.5, 4.5, 5.5, -6.5, 0.0]
                         * 2, np.float32), (2, 8))
    yield "ties", t
    yield "tiny", (rng.standard_normal((4, k)) * 1e-30).astype(np.float32)   # subnormal d
    yield "huge", (rng.standard_normal((4, k)) * 1e35).astype(np.float32)
    # 0 < amax < ~3.7e-37: id = 127 / amax is inf, x * id inf (or NaN for zeros) -> cvtps_epi32's
    # INT_MIN -> -128 after the packs; q8_1's s from the wrapped int32 sum
    u = (rng.standard_normal((4, k)) * 1e-38).astype(np.float32)
    u[:, 32:64] = 0.0
    u[:, 40] = 1e-39
    yield "id_inf", u
    # inf / NaN blocks: the AVX2 amax reduction's operand order decides where a NaN wins
    n = rng.standard_normal((4, k), dtype=np.float32)
    for blk in range(0, k // 32, 3):
        n[blk % 4, 32 * blk + (blk * 7) % 32] = np.nan if blk % 2 else np.inf
    n[1, 5] = -np.inf
    n[2, 0:32] = np.nan
    yield "nonfinite", n


@pytest.mark.parametrize("t", Q8, ids=["q8_0", "q8_1"])
def test_host_quantize_matches_avx2_oracle(t):
    rng = np.random.default_rng(123)
    for name, x in cases(rng):
        got = host_quant(t, x)
        want = ORACLE.quantize(t, x, ol.QUANT_AVX)
        assert np.array_equal(got, want), name


def test_host_quantize_errors():
    x = np.zeros(64, np.float32)
    y = np.zeros(256, np.uint8)
    xp, yp = x.ctypes.data_as(ctypes.c_void_p), y.ctypes.data_as(ctypes.c_void_p)
    assert la.lib.lamm_hip_quantize_host(ol.Q4_0, xp, yp, ctypes.c_int64(64)) == 1      # LAMM_ERR_TYPE
    assert la.lib.lamm_hip_quantize_host(ol.Q8_0, xp, yp, ctypes.c_int64(48)) == 2      # LAMM_ERR_SHAPE
    assert la.lib.lamm_hip_quantize_host(ol.Q8_0, xp, yp, ctypes.c_int64(0)) == 0


def test_host_quantize_rate():
    """Reported, not asserted: one thread's rate on a prefill activation (512 x 4096 F32)."""
    x = np.random.default_rng(1).standard_normal((512, 4096), dtype=np.float32)
    y = np.zeros(512 * 4096 // 32 * 34, np.uint8)
    dt = 1e9
    for _ in range(3):
        t0 = time.perf_counter()
        rc = la.lib.lamm_hip_quantize_host(ol.Q8_0, x.ctypes.data_as(ctypes.c_void_p),
                                           y.ctypes.data_as(ctypes.c_void_p), ctypes.c_int64(x.size))
        dt = min(dt, time.perf_counter() - t0)
        assert rc == 0
    print(f"host q8_0 quantize: {x.nbytes / dt / 1e9:.2f} GB/s of F32 on one thread")


EDGE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "quant", "edge.npz")


@pytest.mark.parametrize("t", Q8, ids=["q8_0", "q8_1"])
def test_quantizers_match_reference_on_edge_inputs(t):
    """The REAL reference's AVX2 from_float bytes (tools/gen_golden_quant.py: ref_driver_lamm3 quant)
    on id = inf blocks, denormals, inf / NaN at every lane position: the oracle's restatement and the
    host quantizer reproduce them byte for byte."""
    z = np.load(EDGE, allow_pickle=False)
    x, want = z["x"], z[ol.NAMES[t]]
    assert np.array_equal(ORACLE.quantize(t, x, ol.QUANT_AVX), want)
    assert np.array_equal(host_quant(t, x), want)
