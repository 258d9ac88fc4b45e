#!/usr/bin/env python3
"""fp6 prefill GEMM, stationary weights: split-K over 256x128 tiles (LAMM_FP6_SUB=0) vs 128x64
workgroup tiles with K-groups (1: 4 groups of 64x64 waves, 2: 2 groups of 32x64 waves), on
config 3 (4096x512x4096, one slice and four) and the Llama-7B prefill shapes (N=512: q/k/v/o
4096x4096, gate/up 11008x4096, down 4096x11008).  hipGraph-replayed whole launches (bench.py's
time_steps), interleaved arms, medians; one JSON line.  ABVAR / ARMS pick another switch."""
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

SHAPES = [("config3_1slice", 4096, 512, 4096, 1), ("config3_4slices", 4096, 512, 4096, 4),
          ("gate_up", 11008, 512, 4096, 1), ("down", 4096, 512, 11008, 1)]
ARMS = os.environ.get("ARMS", "0,1,2").split(",")
ABVAR = os.environ.get("ABVAR", "LAMM_FP6_SUB")   # the switch the arms set (e.g. LAMM_PREP_HSPLIT)


def main():
    ctx = bench.Ctx(torch, la)
    out = {}
    only = os.environ.get("SHAPES")   # comma-separated subset of the shape names
    for name, M, N, K, slices in SHAPES:
        if only and name not in only.split(","):
            continue
        t = la.Q4_0
        gen = torch.Generator(device="cuda")
        gen.manual_seed(5)
        A, arow = bench.make_weights(torch, la, "q4_0", slices, M, K, gen)
        B = bench.make_activations(torch, la, "q4_0", slices * N, K, gen)
        brow = la.row_bytes(la.Q8_0, K)
        C = torch.zeros(slices * N * M, dtype=torch.float32, device="cuda")
        bt = la.Batch(slices, 1, slices, 1, M * arow, slices * M * arow, N * brow, slices * N * brow, 4 * M * N,
                      4 * M * N * slices)
        W = la.Weights(t, A, M, K, ne02=slices, ne03=1, nba2=M * arow, nba3=slices * M * arow)
        res = {a: [] for a in ARMS}
        ref = None
        for rep in range(5):
            for arm in ARMS:
                os.environ[ABVAR] = arm

                def step(i):
                    W.matmul_torch(B, C, N, batch=bt, stream=torch.cuda.current_stream().cuda_stream)

                _, ev, _ = bench.time_steps(ctx, step, 20, 3)
                res[arm].append(ev * 1e6)
                if rep == 0:
                    got = C[:N * M].cpu()
                    if ref is None:
                        ref = got
                    else:   # same sums in another order: agree to fp32 rounding
                        d = ((got - ref).abs() / (ref.abs() + 1e-3)).max().item()
                        res.setdefault("max_rel_diff_vs_arm0", {})[arm] = d
        flops = 2.0 * M * N * K * slices
        out[name] = {a: {"us": round(statistics.median(v), 2),
                         "TOPs": round(flops / statistics.median(v) / 1e6, 1)} for a, v in res.items() if a in ARMS}
        out[name]["rel_diff"] = res.get("max_rel_diff_vs_arm0", {})
        print(name, out[name], flush=True)
        W.close()
        del A, B, C, W
        torch.cuda.empty_cache()
    os.environ.pop(ABVAR, None)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
