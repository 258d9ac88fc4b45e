"""Golden vectors for the AVX2 activation quantizers on edge inputs (id = 127 / amax
infinite, inf / NaN blocks), made by the REAL reference: oracle/_ref/ref_driver_lamm3 quant runs the
lamm3 build's from_float (LC/ggml-quants.c quantize_row_q8_0 / _q8_1, AVX2 branches) on the rows.
Writes tests/golden/quant/edge.npz (inputs, and the reference's bytes per type); the CPU tests pin
the oracle's restatement and the host quantizer to it.  Run here (needs /root/reference's build)."""
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "oracle", "_ref", "ref_driver_lamm3")


def inputs():
    rng = np.random.default_rng(2026)
    K = 1024
    rows = []
    rows.append(rng.standard_normal(K).astype(np.float32))                     # ordinary
    u = (rng.standard_normal(K) * 1e-38).astype(np.float32)                    # id = inf
    u[32:64] = 0.0
    u[40] = 1e-39
    rows.append(u)
    rows.append(np.full(K, 1e-45, np.float32))                                 # denormal min
    n = rng.standard_normal(K).astype(np.float32)                              # NaN / inf at every
    for blk in range(K // 32):                                                 # lane position
        n[32 * blk + blk % 32] = np.nan if blk % 3 else np.inf
    rows.append(n)
    m = rng.standard_normal(K).astype(np.float32)
    m[0:32] = np.nan
    m[64:96] = -np.inf
    m[96] = np.inf
    m[97] = -np.inf
    m[128 + 8] = np.nan                                                        # NaN in the 2nd
    m[160 + 31] = np.nan                                                       # ... and last lane
    rows.append(m)
    rows.append((rng.standard_normal(K) * 3e38).astype(np.float32))            # near overflow
    return np.stack(rows)


def main():
    x = inputs()
    out = {"x": x}
    with tempfile.TemporaryDirectory() as d:
        xf = os.path.join(d, "x.bin")
        x.tofile(xf)
        for t in ("q8_0", "q8_1"):
            of = os.path.join(d, t + ".bin")
            subprocess.run([EXE, "quant", t, str(x.shape[0]), str(x.shape[1]), xf, of], check=True)
            out[t] = np.fromfile(of, np.uint8)
    dst = os.path.join(ROOT, "tests", "golden", "quant", "edge.npz")
    np.savez_compressed(dst, **out)
    print("wrote", dst, {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    sys.exit(main())
