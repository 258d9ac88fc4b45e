#!/usr/bin/env python3
"""Shader clock inside the config-3 fp6 GEMM (Q4_0 x Q8_0 4096x512x4096, stationary weights,
K-group plan): LAMM_GEMM_VARIANT=20+V makes every workgroup's thread 0 write the s_memtime
(shader clock) and s_memrealtime (100 MHz) ticks it spent from entry to the end of the main
loop into C.  Reports, per ablation V (0 production, 1 DMA only, 2 compute only, 4 compute
without fragment reads), the median workgroup's loop time and the clock it ran at."""
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


def main():
    M, N, K = 4096, 512, 4096
    gen = torch.Generator(device="cuda")
    gen.manual_seed(7)
    A, _ = bench.make_weights(torch, la, "q4_0", 1, M, K, gen)
    B = bench.make_activations(torch, la, "q4_0", N, K, gen)
    C = torch.zeros(N * M, dtype=torch.float32, device="cuda")
    W = la.Weights(la.Q4_0, A, M, K)
    out = {}
    for v in (0, 1, 2, 4, 11):
        os.environ["LAMM_GEMM_VARIANT"] = str(20 + v)
        runs = []
        for rep in range(12):
            C.zero_()
            W.matmul_torch(B, C, N)
            torch.cuda.synchronize()
            c = C[:512].cpu().view(256, 2)
            if rep >= 2:
                runs.append(c)
        clk = torch.stack([r[:, 0] for r in runs]).flatten()
        rt = torch.stack([r[:, 1] for r in runs]).flatten()
        us = rt * 0.01
        ghz = clk / (rt * 10.0)
        out[f"V{v}"] = {"loop_us_median": round(statistics.median(us.tolist()), 2),
                        "loop_us_max": round(max(us.tolist()), 2),
                        "clock_GHz_median": round(statistics.median(ghz.tolist()), 3),
                        "clock_GHz_min": round(min(ghz.tolist()), 3)}
        print(f"V{v}", out[f"V{v}"], flush=True)
    os.environ.pop("LAMM_GEMM_VARIANT", None)
    W.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
