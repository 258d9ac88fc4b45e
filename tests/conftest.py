import glob
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
GOLDEN = os.path.join(HERE, "golden")
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(ROOT, "la-llama.cpp_amd"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950); run with -m gpu")


def load_fixture(path):
    """Golden vector set produced by tools/gen_golden.py from the real reference."""
    z = dict(np.load(path, allow_pickle=False))
    M, N, K = int(z["M"]), int(z["N"]), int(z["K"])
    if int(z["type"]) == 0:  # f32: operands are the stored inputs
        inp = np.load(os.path.join(GOLDEN, f"inputs_{M}x{N}x{K}.npz"), allow_pickle=False)
        z["A_q"] = np.frombuffer(inp["A_f32"].tobytes(), dtype=np.uint8)
        z["B_ref"] = np.frombuffer(inp["B_f32"].tobytes(), dtype=np.uint8)
        z["B_avx"] = z["B_ref"]
    z["name"] = os.path.basename(path)[:-4]
    return z


def fixture_paths():
    return sorted(p for p in glob.glob(os.path.join(GOLDEN, "*.npz"))
                  if not os.path.basename(p).startswith("inputs_"))


def load_inputs(M, N, K):
    z = np.load(os.path.join(GOLDEN, f"inputs_{M}x{N}x{K}.npz"), allow_pickle=False)
    return z["A_f32"], z["B_f32"]


def rel_err(c, ref, absdot):
    """|c - ref| / max(|ref|, sum_k |a_k b_k|)  -- SURVEY §8c parity metric."""
    denom = np.maximum(np.abs(ref.astype(np.float64)), absdot.astype(np.float64))
    denom = np.maximum(denom, 1e-30)
    return np.abs(c.astype(np.float64) - ref.astype(np.float64)) / denom
