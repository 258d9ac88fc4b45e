"""One dq16 A/B point: q4_0 (or argv[1]) config 3 forced onto the dq16 engine with whatever
liblamm_hip.so LAMM_HIP_LIB names (tools/build_dq_var.sh probe builds); prints the per-launch time
(hipGraph of 50, best of 5) and, for the clock builds (DQ_AB=3), the first workgroup's shader-clock
and 100 MHz real-time deltas from C[0], C[1] -> its mean clock."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "la-llama.cpp_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import lamm_amd as la  # noqa: E402
from bench import make_weights, make_activations  # noqa: E402

fmt = sys.argv[1] if len(sys.argv) > 1 else "q4_0"
M, N, K = [int(x) for x in (sys.argv[2:5] if len(sys.argv) > 4 else (4096, 512, 4096))]
os.environ["LAMM_GEMM_PATH"] = "dq16"
la.reload_env()
t = la.BY_NAME[fmt]
gen = torch.Generator(device="cuda")
gen.manual_seed(21)
A, rb = make_weights(torch, la, fmt, 1, M, K, gen)
B = make_activations(torch, la, fmt, N, K, gen)
C = torch.zeros(N * M, dtype=torch.float32, device="cuda")
s = torch.cuda.Stream()
reps = 50
with torch.cuda.stream(s):
    la.mul_mat_torch(t, A, B, C, M, N, K, stream=s.cuda_stream)
    s.synchronize()
    clk = C[:2].cpu().tolist()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(reps):
            la.mul_mat_torch(t, A, B, C, M, N, K, stream=s.cuda_stream)
    g.replay()
    s.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(5):
        e0.record(s)
        g.replay()
        e1.record(s)
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / reps)
r = {"lib": os.path.basename(os.environ.get("LAMM_HIP_LIB", "liblamm_hip.so")), "fmt": fmt, "shape": [M, N, K],
     "us": round(best, 3), "TOPs": round(2 * M * N * K / best / 1e6, 1)}
if "clock" in r["lib"]:
    r["wg0_cycles"], r["wg0_rt_ticks"] = clk
    r["wg0_us"] = clk[1] / 100.0
    r["wg0_GHz"] = clk[0] / clk[1] / 10.0 if clk[1] else None
print(json.dumps(r), flush=True)
