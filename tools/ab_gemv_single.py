#!/usr/bin/env python3
"""A/B of decode GEMV kernels (LAMM_GEMV_RPW = waves per workgroup of lamm_gemv_rpw.hip, 0 = the
wave-group kernels of lamm_gemv.hip) in ONE process, interleaved rounds, two workloads:

  single : BASELINE config 2 as the survey states it -- one M x K GEMV per launch, launches
           rotating over enough distinct weight copies (> 256 MiB MALL), event-timed per launch;
  stacked: one launch over S slices (> MALL) -- the steady-state rate;
  single_hot: one weight every call (served from the Infinity Cache) -- what a prefetch buys.

Also each shape with F32 activations (ggml INIT fused).  Checks every variant's C against the
default within 1e-5 relative.  Prints one JSON line (us per launch, TB/s of A + B + C bytes)."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "la-llama.cpp_amd"))
sys.path.insert(0, ROOT)
import lamm_amd as la  # noqa: E402
import bench  # noqa: E402


def timed(fn, reps, stream, graph=True):
    """us per fn call.  graph=True: the reps calls are captured once as a hipGraph and the graph
    is replayed (GPU time per launch, not the host's Python/ctypes submission rate, which is
    ~5 us per call and would otherwise be what a back-to-back loop of short launches measures)."""
    for _ in range(5):
        fn(0)
    torch.cuda.synchronize()
    if graph:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for r in range(reps):
                fn(r)
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / (3 * reps)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for r in range(reps):
        fn(r)
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    variants = (sys.argv[1] if len(sys.argv) > 1 else "0,auto,4,8,16").split(",")
    fmt = os.environ.get("FMT", "q4_0")
    shapes = [tuple(map(int, s.split("x"))) for s in os.environ.get("SHAPES", "4096x4096").split(",")]
    t = la.BY_NAME[fmt]
    vt = la.vec_dot_type(t)
    stream = torch.cuda.current_stream()
    out = {"fmt": fmt, "shapes": {}}
    for (M, K) in shapes:
        u = bench.gemv_bytes(la, fmt, M, K)
        sl = max(8, -(-int(1.15 * bench.MALL_BYTES) // u))
        gen = torch.Generator(device="cuda")
        gen.manual_seed(3)
        A, arow = bench.make_weights(torch, la, fmt, sl, M, K, gen)
        B = bench.make_activations(torch, la, fmt, sl, K, gen)
        X = torch.randn(sl, K, device="cuda", generator=gen)
        kb = K // la.blck_size(t)
        brow = la.row_bytes(vt, K)
        C = torch.zeros(sl * M, dtype=torch.float32, device="cuda")
        Cs = torch.zeros(M, dtype=torch.float32, device="cuda")
        mats = [la.Matrix(A.data_ptr() + z * M * arow, t, M, kb, kb) for z in range(sl)]
        Bm = la.Matrix(B.data_ptr(), vt, kb, 1, kb)
        Xm = la.Matrix(X.data_ptr(), la.F32, K, 1, K)
        Csm = la.Matrix(Cs.data_ptr(), la.F32, M, 1, M)
        Cm = la.Matrix(C.data_ptr(), la.F32, M, 1, M)
        Am = mats[0]
        bt = la.Batch(sl, 1, sl, 1, M * arow, sl * M * arow, brow, sl * brow, 4 * M, 4 * M * sl)
        res = {v: {"single": [], "single_f32": [], "single_hot": [], "single_eager": [], "stacked": []}
               for v in variants}
        outs = {}
        for rnd in range(5):
            for v in variants:
                # "<waves>b": the same with per-lane activation blocks (LAMM_GEMV_LANEB=1)
                os.environ["LAMM_GEMV_LANEB"] = "1" if v.endswith("b") else "0"
                w = v.rstrip("b")
                if w == "auto":
                    os.environ.pop("LAMM_GEMV_RPW", None)
                else:
                    os.environ["LAMM_GEMV_RPW"] = w
                cs = lambda: torch.cuda.current_stream().cuda_stream   # the capture stream inside graphs
                res[v]["single"].append(timed(lambda r: la.matmul(mats[r % sl], Bm, Csm, cs()), 200, stream))
                res[v]["single_f32"].append(timed(lambda r: la.matmul(mats[r % sl], Xm, Csm, cs()), 200, stream))
                # the same weight every call: served from the 256 MiB Infinity Cache (MALL-hot)
                res[v]["single_hot"].append(timed(lambda r: la.matmul(mats[0], Xm, Csm, cs()), 200, stream))
                res[v]["single_eager"].append(timed(lambda r: la.matmul(mats[r % sl], Bm, Csm, cs()), 200, stream, False))
                res[v]["stacked"].append(timed(lambda r: la.matmul_batched(Am, Bm, Cm, bt, cs()), 20, stream))
                if rnd == 0:
                    la.matmul(mats[1], Bm, Csm, stream.cuda_stream)
                    la.matmul(mats[2], Xm, Cm, stream.cuda_stream)
                    torch.cuda.synchronize()
                    outs[v] = (Cs.clone(), C[:M].clone())
        os.environ.pop("LAMM_GEMV_RPW", None)
        os.environ.pop("LAMM_GEMV_LANEB", None)
        summ = {}
        for v in variants:
            d = {}
            for k, arr in res[v].items():
                med = sorted(arr)[len(arr) // 2]
                nbytes = u * (sl if k == "stacked" else 1)
                d[k] = {"us": round(med, 3), "TBs": round(nbytes / (med * 1e-6) / 1e12, 3)}
            ref = outs[variants[0]]
            d["max_rel_vs_first"] = max(float(((o - r).abs().max() / r.abs().max()).item())
                                        for o, r in zip(outs[v], ref))
            summ[v] = d
        out["shapes"][f"{M}x{K}"] = {"slices": sl, "bytes_per_call": u, "variants": summ}
        del A, B, X, C
        torch.cuda.empty_cache()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
