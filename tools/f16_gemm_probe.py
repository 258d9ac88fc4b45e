"""Ballpark of a plain f16 GEMM at config 3's shape (4096 x 512 x 4096) and config 4's, through
torch (hipBLASLt): what a weight-stationary f16 copy of the weights would run at."""
import torch

def t(fn, n=200):
    for _ in range(10): fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3

for (M, N, K) in ((4096, 512, 4096), (11008, 512, 4096), (4096, 512, 11008)):
    for dt in (torch.float16, torch.bfloat16):
        A = torch.randn(M, K, device="cuda", dtype=dt)
        B = torch.randn(N, K, device="cuda", dtype=dt)
        us = t(lambda: torch.matmul(B, A.t()))
        print(f"{M}x{N}x{K} {dt}: {us:.2f} us  {2*M*N*K/us/1e6:.0f} TFLOP/s", flush=True)
    A8 = torch.randn(M, K, device="cuda").to(torch.float8_e4m3fn)
    B8 = torch.randn(N, K, device="cuda").to(torch.float8_e4m3fn)
    one = torch.tensor(1.0, device="cuda")
    try:
        us = t(lambda: torch._scaled_mm(B8, A8.t(), scale_a=one, scale_b=one, out_dtype=torch.float32))
        print(f"{M}x{N}x{K} fp8 scaled_mm: {us:.2f} us  {2*M*N*K/us/1e6:.0f} TFLOP/s", flush=True)
    except Exception as ex:
        print("fp8", str(ex)[:200])
