#!/usr/bin/env python3
"""Config 3 single slice (Q4_0 x Q8_0, M=4096 N=512 K=4096, stationary weights): run the fp6
GEMM under every K-split (LAMM_FP6_SPLIT) and ablation (LAMM_GEMM_VARIANT: 0 production,
1 no compute, 2 no DMA, 3 no epilogue FMAs, 6 no P-MFMA, 7 no S-MFMA) -- 20 eager calls each,
meant to run under `rocprofv3 --kernel-trace` (per-kernel durations by name and grid)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "la-llama.cpp_amd"))
sys.path.insert(0, ROOT)
import lamm_amd as la  # noqa: E402
import bench  # noqa: E402


def main():
    M, N, K = 4096, 512, 4096
    t = la.Q4_0
    gen = torch.Generator(device="cuda")
    gen.manual_seed(7)
    A, arow = bench.make_weights(torch, la, "q4_0", 1, M, K, gen)
    B = bench.make_activations(torch, la, "q4_0", N, K, gen)
    C = torch.zeros(N * M, dtype=torch.float32, device="cuda")
    W = la.Weights(t, A, M, K)
    splits = os.environ.get("SPLITS", "1,2,4,8").split(",")
    variants = os.environ.get("VARIANTS", "0,1,2,3,6,7").split(",")
    preps = os.environ.get("PREPS", "1").split(",")   # LAMM_FP6_PREP_TILED (a removed A/B arm)
    for pr in preps:
        for sp in splits:
            for v in variants:
                os.environ["LAMM_FP6_PREP_TILED"] = pr
                os.environ["LAMM_FP6_SPLIT"] = sp
                os.environ["LAMM_GEMM_VARIANT"] = v
                for _ in range(20):
                    W.matmul_torch(B, C, N)
                torch.cuda.synchronize()
                print(f"prep_tiled {pr} split {sp} variant {v} done", flush=True)
    W.close()


if __name__ == "__main__":
    main()
