"""The drop-in proof: the reference's own, unchanged ggml (llama.cpp-b2430 ggml.c built
from /root/reference with -DLA_LLAMA, its hook LC/ggml.c:10858-10863 resolved to our
include/loongarch_matmul.h, linked against liblamm_hip.so -- oracle/Makefile target
ref_driver_hip) runs ggml_graph_compute(ggml_mul_mat(A, B)) on the golden inputs.  By
default the hook claims INIT and quantizes B on the GPU; with LAMM_HIP_GPU_QUANT=0 ggml's
INIT quantizes it on the CPU as always.  The graph output must match the reference's own
CPU outputs for the same inputs, and both modes must agree bit for bit."""
import os
import subprocess

import numpy as np
import pytest

from conftest import fixture_paths, load_fixture, load_inputs, rel_err

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "oracle", "_ref", "ref_driver_hip")
FIXTURES = fixture_paths()
NAMES = {0: "f32", 2: "q4_0", 3: "q4_1", 6: "q5_0", 7: "q5_1", 8: "q8_0", 10: "q2_k",
         12: "q4_k", 13: "q5_k", 14: "q6_k", 1: "f16"}


@pytest.fixture(scope="module")
def exe():
    if not os.path.exists(EXE):
        pytest.fail(f"{EXE} missing: build it in the build container (make -C oracle ref)")
    return EXE


@pytest.mark.parametrize("path", FIXTURES, ids=[p.rsplit("/", 1)[-1][:-4] for p in FIXTURES])
def test_unchanged_ggml_graph_through_lamm_hip(exe, path, tmp_path):
    z = load_fixture(path)
    t, M, N, K = int(z["type"]), int(z["M"]), int(z["N"]), int(z["K"])
    a, b = load_inputs(M, N, K)
    pa, pb = tmp_path / "a.bin", tmp_path / "b.bin"
    a.tofile(pa)
    b.tofile(pb)
    out = str(tmp_path / "o")
    r = subprocess.run([exe, "gen", NAMES[t], str(M), str(N), str(K), "4", str(pa), str(pb), out],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert np.array_equal(np.fromfile(out + ".A.bin", np.uint8), z["A_q"])
    c = np.fromfile(out + ".C.bin", np.float32).reshape(N, M)
    # the hook computed all M rows (no M % nth drop) and matches the reference CPU paths
    assert np.isfinite(c).all()
    assert rel_err(c, z["C_vdot_avx"], z["absdot"]).max() < 1e-3
    # the CPU-INIT mode (the reference's own flow) gives the same bytes
    out0 = str(tmp_path / "o0")
    r = subprocess.run([exe, "gen", NAMES[t], str(M), str(N), str(K), "4", str(pa), str(pb), out0],
                       capture_output=True, text=True, timeout=120, env=dict(os.environ, LAMM_HIP_GPU_QUANT="0"))
    assert r.returncode == 0, r.stderr[-2000:]
    np.testing.assert_array_equal(np.fromfile(out0 + ".C.bin", np.float32).reshape(N, M), c)
