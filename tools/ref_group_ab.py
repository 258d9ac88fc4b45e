#!/usr/bin/env python3
"""Throughput of the reference-order decode GEMVs as llama.cpp's decode runs them through the
boundary (q8_0 activation row, LAMM_ORDER_REFERENCE): one weight (wo 4096 x 4096, down 4096 x 11008)
and the sibling groups (wq + wk + wv, gate + up: lamm_hip_matmul_group), HIP events over 200
back-to-back launches, weights resident.  A/B of library builds via LAMM_HIP_LIB.
Usage: LAMM_HIP_LIB=path python3 tools/ref_group_ab.py [tag]"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "la-llama.cpp_amd"))
import lamm_amd as la  # noqa: E402

Q4_0, Q8_0 = 2, 8


def weight(M, K, g):
    kb = K // 32
    raw = torch.randint(0, 256, (M * kb * 18 + 64,), dtype=torch.uint8, generator=g)
    a = raw.cuda()
    v = a[:M * kb * 18].view(M * kb, 18)
    v[:, 0] = 0x00
    v[:, 1] = 0x20   # d = 2^-7 (f16 0x2000): finite scales
    return a, la.Matrix(a.data_ptr(), Q4_0, M, kb, kb)


def act(K, g):
    kb = K // 32
    raw = torch.randint(0, 256, (kb * 34,), dtype=torch.uint8, generator=g).cuda()
    v = raw.view(kb, 34)
    v[:, 0] = 0x00
    v[:, 1] = 0x20
    return raw, la.Matrix(raw.data_ptr(), Q8_0, kb, 1, kb)


def time_us(fn, n=100, reps=5):
    """GPU time per launch: n launches captured into one hipGraph (the host's per-call cost out of
    the way), the graph replayed `reps` times, the median replay / n"""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        with torch.cuda.graph(gr, stream=side):
            for _ in range(n):
                fn()
    torch.cuda.synchronize()
    gr.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(reps):
        e0.record()
        gr.replay()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / n)
    return round(sorted(ts)[len(ts) // 2], 2)


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else os.environ.get("LAMM_HIP_LIB", "default")
    g = torch.Generator().manual_seed(1)
    keep, out = [], {"tag": tag}
    for name, Ms, K in (("wo", (4096,), 4096), ("down", (4096,), 11008), ("qkv", (4096,) * 3, 4096),
                        ("gate_up", (11008,) * 2, 4096)):
        ws = [weight(M, K, g) for M in Ms]
        b, Bm = act(K, g)
        Cs = [torch.empty(M, dtype=torch.float32, device="cuda") for M in Ms]
        Cms = [la.Matrix(c.data_ptr(), la.F32, M, 1, M) for c, M in zip(Cs, Ms)]
        As = [w[1] for w in ws]
        keep += [ws, b, Cs]
        cur = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731  (the capture stream inside)
        if len(As) == 1:
            fn = lambda: la.matmul_ex(As[0], Bm, Cms[0], None, la.ORDER_REFERENCE, cur())  # noqa: E731
        else:
            fn = lambda: la.matmul_group(As, Bm, Cms, la.ORDER_REFERENCE, cur())  # noqa: E731
        us = time_us(fn)
        mb = sum(M * (K // 32) * 18 for M in Ms) / 1e6
        out[name] = {"us": us, "TBs": round(mb / us, 3)}
        out[name + "_sum"] = float(np.float64(sum(float(c.double().sum()) for c in Cs)))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
