"""A/B of the int8 K-group engine (LAMM_I8KV=1, no activation prep) against the fp6 engine on
bench.py's config3_gemm (stationary weights, whole launch graph-replayed), one process per setting,
alternating.  python tools/i8kv_ab.py [fmt] [pairs]"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
fmt = sys.argv[1] if len(sys.argv) > 1 else "q4_0"
pairs = int(sys.argv[2]) if len(sys.argv) > 2 else 2
CODE = f"""
import sys, json
sys.path.insert(0, {ROOT!r}); sys.path.insert(0, {os.path.join(ROOT, 'la-llama.cpp_amd')!r})
import torch, lamm_amd as la, bench
ctx = bench.Ctx(torch, la)
per, kern, _, _ = bench.config3_gemm(ctx, {fmt!r}, 4096, 512, 4096, 1, 200)
print(json.dumps({{"whole_us": round(per * 1e6, 2), "kern_us": round(kern * 1e6, 2) if kern else None}}))
"""
for i in range(pairs):
    for v in ("0", "1") if i % 2 == 0 else ("1", "0"):
        env = dict(os.environ, LAMM_I8KV=v)
        r = subprocess.run([sys.executable, "-c", CODE], env=env, capture_output=True, text=True, timeout=300)
        line = r.stdout.strip().splitlines()[-1] if r.returncode == 0 and r.stdout.strip() else r.stderr[-400:]
        print(json.dumps({"fmt": fmt, "i8kv": int(v), "run": i, "result": line}), flush=True)
        if r.returncode != 0:
            sys.exit(r.returncode)
