#!/usr/bin/env python3
"""roofline_trace.py -- the config-2 GEMV kernel timed by the kernel tracer, one dispatch at a time.

bench.py's roofline divides config 2's algorithmic bytes by the kernel's per-launch time from HIP
events over 1000 back-to-back hipGraph-replayed launches.  Under `rocprofv3 --kernel-trace`,
back-to-back dispatches are stretched by the tracer itself (~1 us each: start-to-start equals the
traced duration, profiles/r04/roofline_trace/): its per-dispatch cost is folded into every
duration.  This workload issues the same launches -- bench.py's weights (33 copies > MALL, the same
seeds), activation and C, lamm_hip_matmul from C -- each after the previous one has completed and
the device has idled `--gap-us`, so the tracer times every dispatch on its own.  Run it under
rocprofv3 --kernel-trace --stats (tools/roofline_trace.sh); tools/kt_roofline.py reduces the trace.
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "la-llama.cpp_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--launches", type=int, default=300)
    ap.add_argument("--gap-us", type=float, default=2.0)
    ap.add_argument("--sync-each", action="store_true", help="synchronize after every launch (device idles)")
    ap.add_argument("--fmt", default="q4_0")
    args = ap.parse_args()
    import torch
    import lamm_amd as la
    import bench

    fmt, M, K = args.fmt, 4096, 4096
    t = la.BY_NAME[fmt]
    vt = la.vec_dot_type(t)
    kb = K // la.blck_size(t)
    arow = la.row_bytes(t, K)
    slab = M * arow
    R = max(8, -(-int(1.15 * bench.MALL_BYTES) // slab))
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
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libsteps_loop.so"))
    lib.lamm_steps_matmul_paced.argtypes = [ctypes.POINTER(la.Matrix), ctypes.c_int, ctypes.POINTER(la.Matrix),
                                            ctypes.POINTER(la.Matrix), ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                            ctypes.c_double, ctypes.c_int]
    st = torch.cuda.Stream()
    torch.cuda.synchronize()
    rc = lib.lamm_steps_matmul_paced(mats, R, ctypes.byref(Bm), ctypes.byref(Cm), 0, args.launches,
                                     ctypes.c_void_p(st.cuda_stream), args.gap_us, int(args.sync_each))
    torch.cuda.synchronize()
    assert rc == 0, rc
    print(f"roofline_trace: {args.launches} paced {fmt} {M}x1x{K} launches over {R} weight copies, "
          f"gap {args.gap_us} us{' after a synchronize' if args.sync_each else ''}, engine {la.gemm_engine(fmt, M, 1, K)}")


if __name__ == "__main__":
    main()
