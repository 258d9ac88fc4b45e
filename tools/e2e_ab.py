"""Config 5 through the unchanged llama.cpp with alternating LAMM_* settings: one JSON line per
(repetition, setting), so box drift hits every setting alike.
Usage: python3 tools/e2e_ab.py '{"base": {}, "ksig": {"LAMM_HIP_KERNEL_SIGNAL": "1"}}' [threads] [n_prompt] [reps]"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from bench import llama_e2e  # noqa: E402

settings = json.loads(sys.argv[1])
threads = int(sys.argv[2]) if len(sys.argv) > 2 else 16
n_prompt = int(sys.argv[3]) if len(sys.argv) > 3 else 512
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 2
for rep in range(reps):
    for name, env in settings.items():
        d = llama_e2e(None, n_prompt=n_prompt, n_gen=128, threads=threads, extra_env=env, timeout=300)
        keep = {k: d.get(k) for k in ("pp_tok_s", "tg_tok_s", "tg_from_empty_tok_s", "error") if k in d}
        print(json.dumps({"setting": name, "rep": rep, "threads": threads, "n_prompt": n_prompt, **keep}), flush=True)
