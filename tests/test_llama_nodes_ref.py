"""The node-level parity checker (tests/llama_nodes.py) pinned on the reference itself: the
reference's own llama.cpp-b2430 + lamm opt-3 AVX2 build (oracle/_ref/llama_e2e_lamm3) dumps the
mul_mat nodes of a 2-layer model (--dump-mm) and every node must match the oracle's recompute from
its own operands -- so the GPU test's bar (tests/test_gpu_llama_e2e.py) measures the HIP build, not
the dump or the recompute.  CPU only."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CPU = os.path.join(ROOT, "oracle", "_ref", "llama_e2e_lamm3")


@pytest.mark.skipif(not os.path.exists(CPU), reason="reference build absent (oracle/Makefile ref)")
def test_reference_build_nodes_match_oracle(tmp_path):
    import llama_nodes as ln
    model = str(tmp_path / "synth2.gguf")
    subprocess.run([CPU, "-m", model, "--layers", "2", "--write-only"], check=True, timeout=120,
                   capture_output=True)
    d = tmp_path / "mm"
    d.mkdir()
    r = subprocess.run([CPU, "-m", model, "-t", "8", "-p", "32", "-n", "1", "--dump-mm", str(d)],
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    res = ln.check_nodes(str(d), workers=min(8, os.cpu_count() or 1))
    kinds = {r[2] for r in res}
    assert kinds == {"wq", "wk", "wv", "wo", "w1", "w2", "w3", "KQ", "KQV", "output"}
    assert len(res) == 38
    # the reference's AVX2 float order against the oracle's scalar one: rounding only
    assert max(r[5] for r in res) < 1e-6
    # and bit for bit the oracle's restatement of that order (q4_0 projections, the q6_K output,
    # and the F16 attention nodes KQ / KQV in ggml_vec_dot_f16's AVX2 order): every node
    assert all(r[6] for r in res) and sum(r[6] is not None for r in res) == 38
