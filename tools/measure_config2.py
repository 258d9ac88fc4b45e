#!/usr/bin/env python3
"""measure_config2.py -- how the config-2 numbers depend on the way the steps are issued.

Config 2 (one q4_0 x q8_0 4096x4096 GEMV per step, R > MALL rotated weight copies), each mode
timed like bench.py's timed region (synchronize, wall clock, synchronize) and with HIP events:
  graph<K>   : the K steps captured as one hipGraph, replayed (bench.py round 3)
  cloop<K>   : K lamm_hip_matmul calls issued by a C loop (tools/libsteps_loop.so)
  eager<K>   : K la.matmul calls from Python
Per-launch kernel time:
  b2b        : 1000 back-to-back launches in one graph, events / 1000 (round 3's roofline)
  spaced     : launches separated by a host synchronize, an event pair around each
Run it under `rocprofv3 --kernel-trace --stats` to compare the tracer's per-dispatch durations
with each mode (the phases run in the order printed; --phase picks one).
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "la-llama.cpp_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--phase", default="all")
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import torch
    import lamm_amd as la
    import bench

    fmt, M, K = "q4_0", 4096, 4096
    t = la.BY_NAME[fmt]
    vt = la.vec_dot_type(t)
    kb = K // 32
    arow = la.row_bytes(t, K)
    slab = M * arow
    R = 33
    A = torch.empty(R * slab + 64, dtype=torch.uint8, device="cuda")
    for c in range(R):
        g = torch.Generator(device="cuda")
        g.manual_seed(1000 + c)
        full, _ = bench.make_weights(torch, la, fmt, 1, M, K, g)
        A[c * slab:(c + 1) * slab] = full
    g = torch.Generator(device="cuda")
    g.manual_seed(7)
    B = bench.make_activations(torch, la, fmt, 1, K, g)
    C = torch.zeros(M, dtype=torch.float32, device="cuda")
    mats = (la.Matrix * R)(*[la.Matrix(A.data_ptr() + c * slab, t, M, kb, kb) for c in range(R)])
    Bm = la.Matrix(B.data_ptr(), vt, kb, 1, kb)
    Cm = la.Matrix(C.data_ptr(), la.F32, M, 1, M)
    unit = bench.gemv_bytes(la, fmt, M, K)
    steps_lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libsteps_loop.so"))
    steps_lib.lamm_steps_matmul.argtypes = [ctypes.POINTER(la.Matrix), ctypes.c_int, ctypes.POINTER(la.Matrix),
                                            ctypes.POINTER(la.Matrix), ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    st = torch.cuda.Stream()
    sp = st.cuda_stream
    out = {}

    def timed(fn):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record(st)
        fn()
        e1.record(st)
        torch.cuda.synchronize()
        return time.perf_counter() - t0, e0.elapsed_time(e1) * 1e-3

    def rec(name, vals, steps):
        w = sorted(v[0] for v in vals)[len(vals) // 2] / steps
        e = sorted(v[1] for v in vals)[len(vals) // 2] / steps
        out[name] = {"wall_us_per_step": round(w * 1e6, 3), "event_us_per_step": round(e * 1e6, 3),
                     "value_GBs": round(unit / w / 1e9, 1)}
        print(name, out[name], flush=True)

    with torch.cuda.stream(st):
        for i in range(5):
            la.matmul(mats[i % R], Bm, Cm, sp)
    torch.cuda.synchronize()
    for K_ in (20, 200):
        if args.phase in ("all", "graph"):
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr, stream=st):
                for s in range(K_):
                    la.matmul(mats[s % R], Bm, Cm, torch.cuda.current_stream().cuda_stream)
            gr.replay()
            torch.cuda.synchronize()
            rec(f"graph{K_}", [timed(gr.replay) for _ in range(args.reps)], K_)
            del gr
        if args.phase in ("all", "cloop"):
            rec(f"cloop{K_}", [timed(lambda: steps_lib.lamm_steps_matmul(mats, R, ctypes.byref(Bm), ctypes.byref(Cm),
                                                                         0, K_, ctypes.c_void_p(sp)))
                               for _ in range(args.reps)], K_)
        if args.phase in ("all", "eager"):
            def eager():
                for s in range(K_):
                    la.matmul(mats[s % R], Bm, Cm, sp)
            rec(f"eager{K_}", [timed(eager) for _ in range(args.reps)], K_)
    if args.phase in ("all", "b2b"):
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr, stream=st):
            for s in range(1000):
                la.matmul(mats[s % R], Bm, Cm, torch.cuda.current_stream().cuda_stream)
        gr.replay()
        torch.cuda.synchronize()
        rec("b2b1000", [timed(gr.replay) for _ in range(3)], 1000)
        del gr
    if args.phase in ("all", "spaced"):
        ds = []
        for s in range(300):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            la.matmul(mats[s % R], Bm, Cm, sp)
            e1.record(st)
            torch.cuda.synchronize()
            ds.append(e0.elapsed_time(e1) * 1e3)
        ds.sort()
        out["spaced"] = {"median_us": round(ds[len(ds) // 2], 3), "mean_us": round(sum(ds) / len(ds), 3),
                         "min_us": round(ds[0], 3)}
        print("spaced", out["spaced"], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
