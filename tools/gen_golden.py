#!/usr/bin/env python3
"""Generate tests/golden/*.npz from the REAL reference (run in the build container only).

Test infrastructure: needs oracle/_ref/ref_driver_{scalar,lamm3} (oracle/Makefile
builds them out-of-tree from /root/reference).  For every (format, shape) it feeds the
same seeded N(0,1) float32 inputs to

  * the scalar ggml build  -> A_q (ggml_quantize_chunk), B_ref (from_float_reference),
                              C_scalar (graph mul_mat = stock scalar vec_dot)
  * the AVX2 lamm3 build   -> B_avx (from_float, AVX2 quantizer used in INIT),
                              C_lamm3 (graph mul_mat through lamm_mul_mat, opt level 3),
                              C_vdot_avx (stock AVX2 vec_dot on B_avx, row by row)

and stores them with the fp64 dot of the dequantized operands.  Inputs are regenerated
from `seed` by numpy (PCG64); the sha256 of the inputs is stored so a drifting RNG is
detected instead of silently producing wrong comparisons.

Usage:  python tools/gen_golden.py  [--out tests/golden]
"""
import argparse
import ctypes
import hashlib
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(ROOT, "oracle", "_ref")

FORMATS = {  # name -> (ggml type id, vec_dot type id)
    "f32": (0, 0), "q4_0": (2, 8), "q4_1": (3, 9), "q5_0": (6, 8),
    "q5_1": (7, 9), "q8_0": (8, 8), "q2_k": (10, 15),
    # SURVEY §8f "next" formats (not lamm's: the reference routes them to stock ggml, so
    # C_lamm3 is ggml's own AVX2 vec_dot there)
    "q4_k": (12, 15), "q5_k": (13, 15), "q6_k": (14, 15), "f16": (1, 1),
}
# (M, N, K): tile remainders; the reference's own LAMM_DEBUG shape
# (src/la-benchmark-matmult.cpp:176-178); a decode-shaped GEMV.
SHAPES = [(67, 9, 512), (33, 18, 4096), (16, 1, 4096)]


def inputs(seed, M, N, K):
    rng = np.random.default_rng(seed)
    a = rng.standard_normal((M, K), dtype=np.float32)
    b = rng.standard_normal((N, K), dtype=np.float32)
    return a, b


def sha(a, b):
    return hashlib.sha256(a.tobytes() + b.tobytes()).hexdigest()


def run_gen(binary, fmt, M, N, K, a, b, tmp):
    pa, pb = os.path.join(tmp, "a.bin"), os.path.join(tmp, "b.bin")
    a.tofile(pa)
    b.tofile(pb)
    pre = os.path.join(tmp, os.path.basename(binary))
    subprocess.run([binary, "gen", fmt, str(M), str(N), str(K), "4", pa, pb, pre], check=True)
    rd = lambda s, dt=np.uint8: np.fromfile(pre + s, dtype=dt)
    return dict(A=rd(".A.bin"), Bq=rd(".Bq.bin"), Br=rd(".Br.bin"),
                C=rd(".C.bin", np.float32).reshape(N, M), Cv=rd(".Cv.bin", np.float32).reshape(N, M))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "tests", "golden"))
    ap.add_argument("--formats", default=",".join(FORMATS), help="comma-separated subset")
    args = ap.parse_args()
    wanted = args.formats.split(",")
    os.makedirs(args.out, exist_ok=True)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib  # our restatement, used only for the fp64 dequantized reference
    lo = oracle_lib.Oracle()

    for si, (M, N, K) in enumerate(SHAPES):   # inputs stored once per shape
        a, b = inputs(1000 + 17 * si, M, N, K)
        np.savez_compressed(os.path.join(args.out, f"inputs_{M}x{N}x{K}.npz"), A_f32=a, B_f32=b,
                            seed=np.int64(1000 + 17 * si), input_sha256=np.array(sha(a, b)))
    with tempfile.TemporaryDirectory() as tmp:
        for fmt, (t, vt) in FORMATS.items():
            if fmt not in wanted:
                continue
            for si, (M, N, K) in enumerate(SHAPES):
                seed = 1000 + 17 * si
                a, b = inputs(seed, M, N, K)
                sc = run_gen(os.path.join(REF, "ref_driver_scalar"), fmt, M, N, K, a, b, tmp)
                l3 = run_gen(os.path.join(REF, "ref_driver_lamm3"), fmt, M, N, K, a, b, tmp)
                assert np.array_equal(sc["A"], l3["A"]), f"{fmt}: A quantization differs between builds"
                # fp64 dequantized reference (for information / normalisation only)
                Ad = lo.dequantize(t, sc["A"], M, K).astype(np.float64)
                Bd = lo.dequantize(vt, sc["Br"], N, K).astype(np.float64)
                C64 = (Bd @ Ad.T).astype(np.float64)           # [N][M]
                absdot = (np.abs(Bd) @ np.abs(Ad).T)           # sum_k |a_k b_k|
                name = os.path.join(args.out, f"{fmt}_{M}x{N}x{K}.npz")
                np.savez_compressed(
                    name, type=np.int32(t), vdt=np.int32(vt), M=np.int32(M), N=np.int32(N),
                    K=np.int32(K), seed=np.int64(seed), input_sha256=np.array(sha(a, b)),
                    # f32: operands are the stored inputs themselves (inputs_*.npz)
                    **({} if t == 0 else dict(A_q=sc["A"], B_ref=sc["Br"], B_avx=l3["Bq"])),
                    C_scalar=sc["C"], C_lamm3=l3["C"], C_vdot_avx=l3["Cv"],
                    C_fp64=C64, absdot=absdot,
                    )
                print(f"wrote {name} ({os.path.getsize(name)} B)")


if __name__ == "__main__":
    main()
