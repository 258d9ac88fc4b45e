#!/usr/bin/env python3
"""Weight quantizer speed (lamm_hip_quantize on weight types): a 32000 x 4096 F32 matrix (the
Llama output.weight shape) into each format, event-timed over 5 calls."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "la-llama.cpp_amd"))
import lamm_amd as la  # noqa: E402

M, K = 32000, 4096
x = torch.randn(M, K, device="cuda")
out = {}
for name in ("q4_0", "q2_k", "q4_k", "q5_k", "q6_k"):
    t = la.BY_NAME[name]
    y = torch.zeros(la.row_bytes(t, K) * M + 64, dtype=torch.uint8, device="cuda")
    la.quantize_torch(t, x, y, flavour=0)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        la.quantize_torch(t, x, y, flavour=0)
    e1.record()
    torch.cuda.synchronize()
    out[name] = round(e0.elapsed_time(e1) / 5, 3)
print(json.dumps({"shape": [M, K], "ms_per_call": out}))
