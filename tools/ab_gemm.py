#!/usr/bin/env python3
"""Interleaved A/B timing of GEMM variants (LAMM_GEMM_VARIANT) in ONE process.

Variants: "fp6" = the block-scaled fp6 GEMM (production for q4_0/q4_1/q5_0), "i8" = the
MFMA-i8 GEMM (LAMM_GEMM_PATH=i8); integers select ablations of the i8 kernel
(LAMM_GEMM_VARIANT: 1 = no MFMA phase, 2 = no weight unpack, 3 = no DMA, 4 = prep pass only)."""
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
    variants = (sys.argv[1] if len(sys.argv) > 1 else "fp6,i8").split(",")
    fmt = os.environ.get("FMT", "q4_0")
    M, K, N = 4096, 4096, int(os.environ.get("NCOL", "512"))
    slices = int(os.environ.get("SLICES", "4"))
    t = la.BY_NAME[fmt]
    vt = la.vec_dot_type(t)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(7)
    A, arow = bench.make_weights(torch, la, fmt, slices, M, K, gen)
    B = bench.make_activations(torch, la, fmt, slices * N, K, gen)
    kb = K // la.blck_size(t)
    brow = la.row_bytes(vt, K)
    res = {v: [] for v in variants}
    stream = torch.cuda.current_stream()
    C = torch.zeros(slices * N * M, dtype=torch.float32, device="cuda")
    Am = la.Matrix(A.data_ptr(), t, M, kb, kb)
    Bm = la.Matrix(B.data_ptr(), vt, kb, N, kb)
    Cm = la.Matrix(C.data_ptr(), la.F32, M, N, M)
    bt = la.Batch(slices, 1, slices, 1, M * arow, slices * M * arow, N * brow, slices * N * brow,
                  4 * M * N, 4 * M * N * slices)
    W = None
    if os.environ.get("STATIONARY") == "1":   # weights as a lamm_hip_weights handle (packed once)
        W = la.Weights(t, A, M, K, ne02=slices, ne03=1, nba2=M * arow, nba3=slices * M * arow)

    def run():
        if W is not None:
            W.matmul_torch(B, C, N, batch=bt, stream=stream.cuda_stream)
        else:
            la.matmul_batched(Am, Bm, Cm, bt, stream.cuda_stream)
    for rnd in range(5):
        for v in variants:
            os.environ.pop("LAMM_FP6_WJ", None)
            os.environ.pop("LAMM_FP6_SPLIT", None)
            if v.startswith("fp6s"):     # fp6 with a forced K-split count: fp6s4
                os.environ["LAMM_GEMM_PATH"] = "fp6"
                os.environ["LAMM_GEMM_VARIANT"] = "0"
                os.environ["LAMM_FP6_SPLIT"] = v[4:]
            elif v in ("fp6", "i8"):
                os.environ["LAMM_GEMM_PATH"] = v
                os.environ["LAMM_GEMM_VARIANT"] = "0"
            elif v.startswith("fp6w"):   # fp6 wave-tile width: fp6w1 = 16 waves of 32x64
                os.environ["LAMM_GEMM_PATH"] = "fp6"
                os.environ["LAMM_GEMM_VARIANT"] = "0"
                os.environ["LAMM_FP6_WJ"] = v[4:]
            elif v.startswith("fp6-"):   # fp6 ablations: fp6-1 no compute, fp6-2 no DMA, fp6-3 no FMAs
                os.environ["LAMM_GEMM_PATH"] = "fp6"
                os.environ["LAMM_GEMM_VARIANT"] = v[4:]
            else:
                os.environ["LAMM_GEMM_PATH"] = "i8"
                os.environ["LAMM_GEMM_VARIANT"] = v
            for _ in range(2):
                run()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(10):
                run()
            e1.record(stream)
            torch.cuda.synchronize()
            res[v].append(e0.elapsed_time(e1) * 1e3 / 10)
    # cross-check: the fp6 and i8 engines must agree (both compute exact block dots)
    outs = {}
    for v in ("fp6", "i8"):
        os.environ["LAMM_GEMM_PATH"] = v
        os.environ["LAMM_GEMM_VARIANT"] = "0"
        C.fill_(float("nan"))
        la.matmul_batched(Am, Bm, Cm, bt, stream.cuda_stream)
        torch.cuda.synchronize()
        outs[v] = C.clone()
    diff = ((outs["fp6"] - outs["i8"]).abs() / (outs["i8"].abs() + 1e-3)).max().item()
    flops = 2.0 * M * N * K * slices
    summary = {}
    for v in variants:
        med = sorted(res[v])[len(res[v]) // 2]
        summary[v] = {"median_us": round(med, 2), "TOPs": round(flops / (med * 1e-6) / 1e12, 1)}
    print(json.dumps({"fmt": fmt, "M": M, "N": N, "K": K, "slices": slices, "fp6_vs_i8_max_rel": diff,
                      "variants": summary}))


if __name__ == "__main__":
    main()
