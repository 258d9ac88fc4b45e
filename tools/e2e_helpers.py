"""Config 5 decode through the unchanged llama.cpp at -t 16 and -t 8 with each LAMM_HIP_HELPERS mode
(what ggml's other pool threads do while thread 0 runs a matmul on the GPU): pp512 + tg128, one
line per (threads, mode), alternating so box drift hits every mode alike."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from bench import llama_e2e  # noqa: E402

out = sys.argv[1] if len(sys.argv) > 1 else None
res = []
for rep in range(2):
    for threads in (16, 8):
        for mode in ("0", "1", "2"):
            d = llama_e2e(None, n_prompt=512, n_gen=128, threads=threads, extra_env={"LAMM_HIP_HELPERS": mode},
                          timeout=300)
            d.update({"threads": threads, "helpers": mode, "rep": rep})
            print(json.dumps(d), flush=True)
            res.append(d)
if out:
    json.dump(res, open(out, "w"), indent=1)
