#!/usr/bin/env python3
"""Interleaved A/B timing of GEMV staging variants in ONE process (guide §5.4 rule 24).

Each variant (LAMM_GEMV_VARIANT) runs the batched q4_0 GEMV (R slices > MALL) `iters`
times per round; rounds interleave the variants.  Outputs must be bit-identical."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "la-llama.cpp_amd"))
sys.path.insert(0, ROOT)
import lamm_amd as la  # noqa: E402
import bench  # noqa: E402


def main():
    variants = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "0,1,2,3").split(",")]
    fmt, M, K, N = os.environ.get("FMT", "q4_0"), 4096, 4096, int(os.environ.get("NCOL", "1"))
    t = la.BY_NAME[fmt]
    vt = la.vec_dot_type(t)
    unit = bench.gemv_bytes(la, fmt, M, K, N)
    slices = max(8, -(-int(1.15 * bench.MALL_BYTES) // unit))
    gen = torch.Generator(device="cuda")
    gen.manual_seed(7)
    A, arow = bench.make_weights(torch, la, fmt, slices, M, K, gen)
    B = bench.make_activations(torch, la, fmt, slices * N, K, gen)
    kb = K // la.blck_size(t)
    brow = la.row_bytes(vt, K)
    outs = {}
    res = {v: [] for v in variants}
    stream = torch.cuda.current_stream()
    for rnd in range(6):
        for v in variants:
            os.environ["LAMM_GEMV_VARIANT"] = str(v)
            C = torch.zeros(slices * N * M, dtype=torch.float32, device="cuda")
            Am = la.Matrix(A.data_ptr(), t, M, kb, kb)
            Bm = la.Matrix(B.data_ptr(), vt, kb, N, kb)
            Cm = la.Matrix(C.data_ptr(), la.F32, M, N, M)
            bt = la.Batch(slices, 1, slices, 1, M * arow, slices * M * arow, N * brow, slices * N * brow,
                          4 * M * N, 4 * M * N * slices)
            for _ in range(3):
                la.matmul_batched(Am, Bm, Cm, bt, stream.cuda_stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(20):
                la.matmul_batched(Am, Bm, Cm, bt, stream.cuda_stream)
            e1.record(stream)
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / 20
            res[v].append(us)
            if rnd == 0:
                outs[v] = C.cpu()
    base = outs[variants[0]]
    summary = {}
    for v in variants:
        med = sorted(res[v])[len(res[v]) // 2]
        summary[v] = {"median_us": round(med, 2), "min_us": round(min(res[v]), 2),
                      "GBs": round(slices * unit / (med * 1e-6) / 1e9, 1),
                      "identical": bool(torch.equal(outs[v], base))}
    print(json.dumps({"fmt": fmt, "N": N, "slices": slices, "variants": summary}))


if __name__ == "__main__":
    main()
