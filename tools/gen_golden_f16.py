#!/usr/bin/env python3
"""Golden vectors for the F16 x F16 attention mul_mats (KQ, KQV) from the REFERENCE itself:
oracle/_ref/llama_e2e_lamm3 (the reference's llama.cpp-b2430 + la-llama.cpp lamm opt-3 AVX2 build,
compiled from /root/reference by oracle/Makefile) runs a 2-layer synthetic Llama-7B-shaped model
(pp40 + 2 decode steps) with --dump-mm, and the layer-0 attention nodes of the prefill and of the
first decode step are kept as they came out of ggml's CPU loop: src0 (the F16 cache view), src1
(F32), dst -- 4 of the 32 heads each, to keep the fixture small.

    python3 tools/gen_golden_f16.py  ->  tests/golden/ref_nodes/f16_attention.npz
"""
import json
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADS = 4


def main():
    exe = os.path.join(ROOT, "oracle", "_ref", "llama_e2e_lamm3")
    if not os.path.exists(exe):
        sys.exit(f"{exe} missing: build oracle/ first (make -C oracle ref)")
    tmp = tempfile.mkdtemp(prefix="lamm_f16_gold_")
    try:
        d = os.path.join(tmp, "dump")
        os.makedirs(d)
        subprocess.run([exe, "-m", os.path.join(tmp, "m.gguf"), "--layers", "2", "--regen", "-t", "8", "-p", "40",
                        "-n", "2", "--dump-mm", d], check=True, capture_output=True)
        with open(os.path.join(d, "index.jsonl")) as f:
            ents = [json.loads(line) for line in f]
        out = {}
        for e in ents:
            if e["src0"] not in ("k-0", "v-0") or e["type0"] != 1:
                continue
            tag = f"{e['phase']}_{'kq' if e['src0'] == 'k-0' else 'kqv'}"
            if tag + "_src0" in out:
                continue
            K, M, ne02, _ = e["ne0"]
            _, N, ne12, _ = e["ne1"]
            a = np.fromfile(os.path.join(d, e["src0_file"]), np.uint16).reshape(ne02, M, K)[:HEADS]
            b = np.fromfile(os.path.join(d, f"{e['idx']}_src1.bin"), np.float32).reshape(ne12, N, K)[:HEADS]
            c = np.fromfile(os.path.join(d, f"{e['idx']}_dst.bin"), np.float32).reshape(ne12, N, M)[:HEADS]
            out[tag + "_src0"], out[tag + "_src1"], out[tag + "_dst"] = a, b, c
            print(tag, "M N K =", M, N, K, "heads kept", HEADS)
        dst = os.path.join(ROOT, "tests", "golden", "ref_nodes", "f16_attention.npz")
        np.savez_compressed(dst, **out)
        print("wrote", dst, os.path.getsize(dst), "bytes")
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
