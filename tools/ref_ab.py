#!/usr/bin/env python3
"""Kernel times of the reference-order paths for an A/B of library builds (LAMM_HIP_LIB): one-column
GEMVs by their dispatch timestamps (lamm_hip_profile_next, median of 200 launches each completed
before the next), prefill GEMMs and the F16 attention by HIP events over 10 back-to-back launches.
Usage: LAMM_HIP_LIB=path python3 tools/ref_ab.py [tag]"""
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "la-llama.cpp_amd"))
sys.path.insert(0, ROOT)
import lamm_amd as la  # noqa: E402
import bench  # noqa: E402


def stream():
    return torch.cuda.current_stream().cuda_stream


def dispatch_us(fn, n=200):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    e1.record()
    torch.cuda.synchronize()
    out = []
    for _ in range(n):
        la.lib.lamm_hip_profile_next(e0._as_parameter_, e1._as_parameter_)
        fn()
        e1.synchronize()
        out.append(e0.elapsed_time(e1) * 1e3)
    return round(statistics.median(out), 2)


def events_us(fn, n=10):
    for _ in range(2):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) * 1e3 / n, 2)


la.lib.lamm_hip_profile_next.argtypes = [__import__("ctypes").c_void_p] * 2
gen = torch.Generator(device="cuda")
gen.manual_seed(7)
out = {"lib": os.environ.get("LAMM_HIP_LIB", "default")}
# REF_AB_ONLY=q4_0: only the 4096 x 4096 q4_0 shapes; REF_AB_SELS=5,6: only these prefill kernels
ONLY = os.environ.get("REF_AB_ONLY")
SELS = tuple(os.environ.get("REF_AB_SELS", "1,2,3,4,5,6").split(","))
for fmt, M, K in (("q4_0", 4096, 4096), ("q4_0", 11008, 4096), ("q4_0", 4096, 11008), ("q4_1", 4096, 4096),
                  ("q5_0", 4096, 4096), ("q5_1", 4096, 4096), ("q6_k", 32000, 4096)):
    if ONLY and (fmt != ONLY or M != 4096 or K != 4096):
        continue
    t = la.BY_NAME[fmt]
    vt = la.vec_dot_type(t)
    A, _ = bench.make_weights(torch, la, fmt, 1, M, K, gen)
    kb = K // la.blck_size(t)
    if fmt != "q6_k":
        x = torch.randn(K, device="cuda", generator=gen)
        C = torch.zeros(M, dtype=torch.float32, device="cuda")
        Am, Bm, Cm = la.Matrix(A.data_ptr(), t, M, kb, kb), la.Matrix(x.data_ptr(), la.F32, K, 1, K), \
            la.Matrix(C.data_ptr(), la.F32, M, 1, M)
        for bpt in ("2", "4"):   # LAMM_REF_GEMV_BPT
            os.environ["LAMM_REF_GEMV_BPT"] = bpt
            out[f"gemv_{fmt}_{M}x{K}_ref{bpt}"] = dispatch_us(
                lambda: la.matmul_ex(Am, Bm, Cm, None, la.ORDER_REFERENCE, stream()))
        os.environ.pop("LAMM_REF_GEMV_BPT")
        out[f"gemv_{fmt}_{M}x{K}_fast"] = dispatch_us(lambda: la.matmul_ex(Am, Bm, Cm, None, 0, stream()))
    N = 512
    x = torch.randn(N, K, device="cuda", generator=gen)
    B = torch.zeros(N * la.row_bytes(vt, K) + 64, dtype=torch.uint8, device="cuda")
    la.quantize_torch(vt, x, B, flavour=1)
    C = torch.zeros(N * M, dtype=torch.float32, device="cuda")
    for v in (SELS if fmt != "q6_k" else ("2",)):
        os.environ["LAMM_REF_MFMA"] = v
        out[f"gemm_{fmt}_{M}x{N}x{K}_ref_mfma{v}"] = events_us(
            lambda: la.mul_mat_torch(t, A, B, C, M, N, K, flags=la.ORDER_REFERENCE))
    os.environ.pop("LAMM_REF_MFMA")
    print(json.dumps(out), flush=True)
for name, M, N, K in (() if ONLY else (("kq", 512, 512, 128), ("kqv", 128, 512, 512))):
    H = 32
    A = (torch.randn(H * M * K, device="cuda", generator=gen) * 0.3).half().view(torch.uint8)
    Bh = torch.randn(H * N * K, device="cuda", generator=gen).half().view(torch.uint8)
    C = torch.zeros(H * N * M, dtype=torch.float32, device="cuda")
    bt = la.Batch(H, 1, H, 1, 2 * M * K, 2 * M * K * H, 2 * N * K, 2 * N * K * H, 4 * M * N, 4 * M * N * H)
    out[f"f16_{name}_ref"] = events_us(lambda: la.mul_mat_torch(la.F16, A, Bh, C, M, N, K, batch=bt,
                                                               flags=la.ORDER_REFERENCE))
print(json.dumps(out), flush=True)
