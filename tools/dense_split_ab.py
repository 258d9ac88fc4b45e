"""Config 1 (F32 512^3, bench.py config1_f32: one call per step, graph replay) under LAMM_DENSE_SPLIT=n,
one process per setting.  python tools/dense_split_ab.py 0 8 16 ..."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CODE = f"""
import sys, json
sys.path.insert(0, {ROOT!r}); sys.path.insert(0, {os.path.join(ROOT, 'la-llama.cpp_amd')!r})
import torch, lamm_amd as la, bench
ctx = bench.Ctx(torch, la)
r = bench.config1_f32(ctx, 200)
print(json.dumps({{"us": r["per_launch_us"], "GFLOPS": r["GFLOPS"], "err": r["max_rel_err_vs_torch_fp32"]}}))
"""
for v in sys.argv[1:] or ["0", "8", "16"]:
    env = dict(os.environ)
    if v != "0":
        env["LAMM_DENSE_SPLIT"] = v
    r = subprocess.run([sys.executable, "-c", CODE], env=env, capture_output=True, text=True, timeout=300)
    line = r.stdout.strip().splitlines()[-1] if r.returncode == 0 and r.stdout.strip() else r.stderr[-400:]
    print(json.dumps({"split": int(v), "result": line}), flush=True)
    if r.returncode != 0:
        sys.exit(r.returncode)
