import sys, json
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/la-llama.cpp_amd')
import torch, lamm_amd as la, bench
ctx = bench.Ctx(torch, la)
for rep in range(3):
    per, kern, _, _ = bench.config3_gemm(ctx, 'q2_k', 4096, 512, 4096, 1, 200)
    print(json.dumps({"fmt": "q2_k", "whole_us": round(per * 1e6, 2), "kern_us": round(kern * 1e6, 2)}), flush=True)
