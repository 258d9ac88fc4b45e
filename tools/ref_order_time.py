#!/usr/bin/env python3
"""Per-launch time of the reference-order kernels (csrc/lamm_ref.hip) against the fast engines on
the shapes the ggml boundary sends them for Llama-7B: decode (N = 1, q8 rows and F32 rows) and
prefill (N = 512) projections, the q6_K output.weight, and the F16 attention mul_mats (KQ, KQV over
32 heads).  HIP events over 20 launches (after 3 warm-up); run it under
`rocprofv3 --kernel-trace --stats` for the kernels' own durations (the events include the Python
call, ~20 us, so short kernels read as that)."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "la-llama.cpp_amd"))
sys.path.insert(0, ROOT)
import lamm_amd as la  # noqa: E402
import bench  # noqa: E402


def timed(fn, n=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


def stream():
    return torch.cuda.current_stream().cuda_stream


out = {}
gen = torch.Generator(device="cuda")
gen.manual_seed(5)
for fmt, M, K, Ns in (("q4_0", 4096, 4096, (1, 512)), ("q4_0", 11008, 4096, (1, 512)), ("q4_0", 4096, 11008, (1, 512)),
                      ("q6_k", 32000, 4096, (1, 512))):
    t = la.BY_NAME[fmt]
    vt = la.vec_dot_type(t)
    A, _ = bench.make_weights(torch, la, fmt, 1, M, K, gen)
    for N in Ns:
        x = torch.randn(N, K, device="cuda", generator=gen)
        B = torch.zeros(N * la.row_bytes(vt, K) + 64, dtype=torch.uint8, device="cuda")
        la.quantize_torch(vt, x, B, flavour=1)
        C = torch.zeros(N * M, dtype=torch.float32, device="cuda")
        res = {"fast_us": round(timed(lambda: la.mul_mat_torch(t, A, B, C, M, N, K)), 2),
               "fast_engine": la.gemm_engine(fmt, M, N, K)}
        variants = ("1", "2", "4") if N > 8 and fmt != "q6_k" else ("",)
        for v in variants:
            os.environ["LAMM_REF_MFMA"] = v or "-1"
            res[f"reference_order_us{('_mfma' + v) if v else ''}"] = round(
                timed(lambda: la.mul_mat_torch(t, A, B, C, M, N, K, flags=la.ORDER_REFERENCE)), 2)
        os.environ.pop("LAMM_REF_MFMA", None)
        if N == 1 and fmt != "q6_k":   # F32 rows: the boundary's decode (quantized in the kernel's staging)
            kb = K // 32
            Am = la.Matrix(A.data_ptr(), t, M, kb, kb)
            Bm = la.Matrix(x.data_ptr(), la.F32, K, 1, K)
            Cm = la.Matrix(C.data_ptr(), la.F32, M, 1, M)
            res["reference_order_f32_rows_us"] = round(
                timed(lambda: la.matmul_ex(Am, Bm, Cm, None, la.ORDER_REFERENCE, stream())), 2)
        out[f"{fmt}_{M}x{N}x{K}"] = res
        print(f"{fmt} {M}x{N}x{K}: {res}", flush=True)

# F16 attention: KQ (n_kv x tokens x head_dim) and KQV (head_dim x tokens x n_kv), 32 heads as slices
for name, M, N, K in (("kq", 512, 512, 128), ("kqv", 128, 512, 512)):
    H = 32
    A = (torch.randn(H * M * K, device="cuda", generator=gen) * 0.3).half()
    Bh = (torch.randn(H * N * K, device="cuda", generator=gen)).half()
    C = torch.zeros(H * N * M, dtype=torch.float32, device="cuda")
    bt = la.Batch(H, 1, H, 1, 2 * M * K, 2 * M * K * H, 2 * N * K, 2 * N * K * H, 4 * M * N, 4 * M * N * H)
    Au, Bu = A.view(torch.uint8), Bh.view(torch.uint8)
    res = {"fast_us": round(timed(lambda: la.mul_mat_torch(la.F16, Au, Bu, C, M, N, K, batch=bt)), 2),
           "reference_order_us": round(timed(lambda: la.mul_mat_torch(la.F16, Au, Bu, C, M, N, K, batch=bt,
                                                                       flags=la.ORDER_REFERENCE)), 2)}
    out[f"f16_{name}_{M}x{N}x{K}x{H}"] = res
    print(f"f16 {name} {M}x{N}x{K} x{H}: {res}", flush=True)
print(json.dumps(out))
