"""A/B of the fp6 weight plane layout (round 6: the affine formats' m beside d in one dword, the last
dword 0, so the P-MFMA takes both planes' pairs without zeroing): config-3-shaped stationary GEMMs
(bench.py config3_gemm: whole launch = activation prep + main kernel, graph replay) for q4_1 / q5_1
(and q4_0, unchanged, as the control), each library in its own process, alternating.
  python tools/aff_ab.py OLD_LIB NEW_LIB [pairs]"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
old, new = sys.argv[1], sys.argv[2]
pairs = int(sys.argv[3]) if len(sys.argv) > 3 else 3
CODE = f"""
import sys, json
sys.path.insert(0, {ROOT!r}); sys.path.insert(0, {os.path.join(ROOT, 'la-llama.cpp_amd')!r})
import torch, lamm_amd as la, bench
ctx = bench.Ctx(torch, la)
out = {{}}
for fmt in ("q4_1", "q5_1", "q4_0"):
    per, kern, _, _ = bench.config3_gemm(ctx, fmt, 4096, 512, 4096, 1, 200)
    out[fmt] = round(per * 1e6, 2)
print(json.dumps(out))
"""
for i in range(pairs):
    for name, lib in (("old", old), ("new", new)) if i % 2 == 0 else (("new", new), ("old", old)):
        env = dict(os.environ, LAMM_HIP_LIB=lib)
        r = subprocess.run([sys.executable, "-c", CODE], env=env, capture_output=True, text=True, timeout=300)
        line = r.stdout.strip().splitlines()[-1] if r.returncode == 0 and r.stdout.strip() else r.stderr[-600:]
        print(json.dumps({"lib": name, "run": i, "whole_us": line}), flush=True)
        if r.returncode != 0:
            sys.exit(r.returncode)
