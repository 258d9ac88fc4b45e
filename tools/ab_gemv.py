#!/usr/bin/env python3
"""Interleaved A/B timing of GEMV kernel variants (LAMM_GEMV_VARIANT) on BASELINE config 2
(q4_0 4096x4096, N=1, 33 slices per launch > MALL) in ONE process; checks every variant's C
against variant 0 bit for bit.  Prints one JSON line (TB/s of algorithmic bytes)."""
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
    variants = (sys.argv[1] if len(sys.argv) > 1 else "0,8,9").split(",")
    fmt = os.environ.get("FMT", "q4_0")
    M = int(os.environ.get("MM", "4096"))
    K = int(os.environ.get("KK", "4096"))
    t = la.BY_NAME[fmt]
    vt = la.vec_dot_type(t)
    u = bench.gemv_bytes(la, fmt, M, K)
    sl = max(8, -(-int(1.15 * bench.MALL_BYTES) // u))
    gen = torch.Generator(device="cuda")
    gen.manual_seed(3)
    A, arow = bench.make_weights(torch, la, fmt, sl, M, K, gen)
    B = bench.make_activations(torch, la, fmt, sl, K, gen)
    kb = K // la.blck_size(t)
    brow = la.row_bytes(vt, K)
    C = torch.zeros(sl * M, dtype=torch.float32, device="cuda")
    Am, Bm, Cm = la.Matrix(A.data_ptr(), t, M, kb, kb), la.Matrix(B.data_ptr(), vt, kb, 1, kb), \
        la.Matrix(C.data_ptr(), la.F32, M, 1, M)
    bt = la.Batch(sl, 1, sl, 1, M * arow, sl * M * arow, brow, sl * brow, 4 * M, 4 * M * sl)
    stream = torch.cuda.current_stream()
    res = {v: [] for v in variants}
    outs = {}
    for rnd in range(7):
        for v in variants:
            os.environ["LAMM_GEMV_VARIANT"] = v
            for _ in range(3):
                la.matmul_batched(Am, Bm, Cm, bt, stream.cuda_stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(20):
                la.matmul_batched(Am, Bm, Cm, bt, stream.cuda_stream)
            e1.record(stream)
            torch.cuda.synchronize()
            res[v].append(e0.elapsed_time(e1) * 1e3 / 20)
            if rnd == 0:
                outs[v] = C.clone()
    os.environ["LAMM_GEMV_VARIANT"] = "0"
    summary = {}
    for v in variants:
        med = sorted(res[v])[len(res[v]) // 2]
        summary[v] = {"median_us": round(med, 2), "TBs": round(sl * u / (med * 1e-6) / 1e12, 3),
                      "equal_to_v0": bool(torch.equal(outs[v], outs[variants[0]]))}
    print(json.dumps({"fmt": fmt, "M": M, "K": K, "slices": sl, "variants": summary}), flush=True)


if __name__ == "__main__":
    main()
