"""Probe of the dequantizing f16 GEMM (lamm_gemm_dq.hip) against the exact engines at BASELINE
config 3's shape for every 32-element format: parity against the oracle on sampled rows (the
north star's bar: |c - c_ref| <= 1e-3 * sum |a b|), and per-launch times (hipGraph of 50 launches,
HIP events) of dq16 / the default exact engine.  Usage: python tools/dq_probe.py [out.json]"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "la-llama.cpp_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import lamm_amd as la  # noqa: E402
import oracle_lib as ol  # noqa: E402
from bench import make_weights, make_activations  # noqa: E402

ORACLE = ol.Oracle()


def run(fmt, M, N, K, path, reps=50):
    if path:
        os.environ["LAMM_GEMM_PATH"] = path
    else:
        os.environ.pop("LAMM_GEMM_PATH", None)
    la.reload_env()
    t = la.BY_NAME[fmt]
    gen = torch.Generator(device="cuda")
    gen.manual_seed(21)
    A, rb = make_weights(torch, la, fmt, 1, M, K, gen)
    B = make_activations(torch, la, fmt, N, K, gen)
    C = torch.zeros(N * M, dtype=torch.float32, device="cuda")
    s = torch.cuda.Stream()
    engine = la.gemm_engine(fmt, M, N, K)
    with torch.cuda.stream(s):
        la.mul_mat_torch(t, A, B, C, M, N, K, stream=s.cuda_stream)
        s.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(reps):
                la.mul_mat_torch(t, A, B, C, M, N, K, stream=s.cuda_stream)
        g.replay()
        s.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        best = 1e9
        for _ in range(5):
            e0.record(s)
            g.replay()
            e1.record(s)
            e1.synchronize()
            best = min(best, e0.elapsed_time(e1) * 1e3 / reps)
    rows = [0, 1, 255, 2048, M - 1]
    vt = la.vec_dot_type(t)
    brow = la.row_bytes(vt, K)
    a = A.view(M, rb)[rows].cpu().numpy()
    b = B[:N * brow].cpu().numpy()
    ref = ORACLE.mul_mat(t, len(rows), N, K, a, b)
    c = C.view(N, M)[:, rows].cpu().numpy()
    Ad = ORACLE.dequantize(t, a, len(rows), K).astype(np.float64)
    Bd = ORACLE.dequantize(vt, b, N, K).astype(np.float64)
    absdot = np.abs(Bd) @ np.abs(Ad).T
    err = np.abs(c - ref) / np.maximum(np.abs(ref), absdot)
    return {"fmt": fmt, "path": path or "default", "engine": engine, "us": round(best, 3),
            "TOPs": round(2 * M * N * K / best / 1e6, 1), "frac_i8": round(2 * M * N * K / best / 1e6 / 5000, 4),
            "max_rel_err": float(err.max()), "mean_rel_err": float(err.mean()), "finite": bool(np.isfinite(c).all())}


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else None
    res = []
    for fmt in ["q4_0", "q8_0", "q4_1", "q5_0", "q5_1"]:
        for path in ["dq16", ""]:
            r = run(fmt, 4096, 512, 4096, path)
            print(json.dumps(r), flush=True)
            res.append(r)
    for (M, N, K) in [(11008, 512, 4096), (4096, 512, 11008), (4096, 128, 4096), (300, 77, 1000)]:
        r = run("q4_0", M, N, K, "dq16") if K % 32 == 0 and (K // 32 * 18) % 16 == 0 else None
        if r is None:
            continue
        r["shape"] = [M, N, K]
        print(json.dumps(r), flush=True)
        res.append(r)
    if out:
        json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
