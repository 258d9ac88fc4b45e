#!/usr/bin/env python3
"""issue_modes.py -- config 2's per-step time by issue mode and step count (round 6): the hipGraph
replay and the library's own AQL queue (bench.py config2_gemv / time_direct), and K lamm_hip_matmul
calls from a C loop (tools/libsteps_loop.so lamm_steps_matmul), at K = 20 (the driver's) and 200,
each timed like bench.py's timed region (caches flushed before it).  JSON lines on stdout."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "la-llama.cpp_amd"))
import torch  # noqa: E402
import lamm_amd as la  # noqa: E402
import bench  # noqa: E402

ctx = bench.Ctx(torch, la)
unit = bench.gemv_bytes(la, "q4_0", 4096, 4096)
lib = bench.steps_lib(la)
lib.lamm_steps_matmul.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(la.Matrix), ctypes.POINTER(la.Matrix),
                                  ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
lib.lamm_steps_graph.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(la.Matrix), ctypes.POINTER(la.Matrix),
                                 ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_float)]
for K in (20, 200, 20, 200):
    g = bench.config2_gemv(ctx, "q4_0", 4096, 4096, K, 5)
    row = {"K": K, "graph_us": round(g["per_step"] * 1e6, 3),
           "direct_us": round(g["direct_step"] * 1e6, 3) if g["direct_step"] else None,
           "kernel_iso_us": round(g["kern"] * 1e6, 3), "read_floor_us": round(g["floor"] * 1e6, 3) if g["floor"] else None}
    # the C loop over the same rotation (its own weights: config2_gemv frees its buffers)
    R = g["R"]
    A = torch.empty(R * 4096 * 2304 + 64, dtype=torch.uint8, device="cuda")
    A.random_(0, 255)
    Bq = bench.make_activations(torch, la, "q4_0", 1, 4096, None)
    C = torch.zeros(4096, dtype=torch.float32, device="cuda")
    mats = (la.Matrix * R)(*[la.Matrix(A.data_ptr() + c * 4096 * 2304, la.Q4_0, 4096, 128, 128) for c in range(R)])
    Bm = la.Matrix(Bq.data_ptr(), la.Q8_0, 128, 1, 128)
    Cm = la.Matrix(C.data_ptr(), la.F32, 4096, 1, 4096)
    st = torch.cuda.Stream()
    lib.lamm_steps_matmul(ctypes.cast(mats, ctypes.c_void_p), R, ctypes.byref(Bm), ctypes.byref(Cm), 0, 5,
                          ctypes.c_void_p(st.cuda_stream))
    bench.flush_caches(torch)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    lib.lamm_steps_matmul(ctypes.cast(mats, ctypes.c_void_p), R, ctypes.byref(Bm), ctypes.byref(Cm), 5, K,
                          ctypes.c_void_p(st.cuda_stream))
    torch.cuda.synchronize()
    row["cloop_us"] = round((time.perf_counter() - t0) / K * 1e6, 3)
    # the same K calls as a hipGraph captured, instantiated and uploaded from C, replayed from C
    out = (ctypes.c_float * 7)()
    rc = lib.lamm_steps_graph(ctypes.cast(mats, ctypes.c_void_p), R, ctypes.byref(Bm), ctypes.byref(Cm), 5, K, 7, out)
    row["cgraph_us"] = round(sorted(out)[3] / K, 3) if rc == 0 else f"rc {rc}"
    row["value_best_GBs"] = round(unit / min(v for k, v in row.items() if k in ("graph_us", "direct_us", "cloop_us", "cgraph_us")
                                            and isinstance(v, float)) / 1e3, 1)
    print(json.dumps(row), flush=True)
    del A, Bq, C
