#!/bin/bash
# config 5 decode / prefill vs ggml thread count and boundary policy (llama.cpp-b2430 + liblamm_hip)
OUT=${1:-gpurun_out/e2e_threads}
mkdir -p "$OUT"
M=${TMPDIR:-/tmp}/lamm_synth_llama7b_q4_0.gguf
timeout -k 10 120 integration/_build/llama_e2e_hip -m "$M" --write-only 2>/dev/null || exit 1
for p in 32 512; do
  for t in 1 2 4 8 16; do
    for v in 0 1; do
      r=$(LAMM_HIP_VIEWS=$v timeout -k 10 300 integration/_build/llama_e2e_hip -m "$M" -t $t -p $p -n 64 2>/dev/null | grep '^{') || exit 1
      echo "p=$p t=$t views=$v $(echo $r | python3 -c 'import sys,json; d=json.load(sys.stdin); print("pp %.1f tok/s  tg %.2f tok/s" % (d["pp_tok_s"], d["tg_tok_s"]))')" | tee -a "$OUT/threads.txt"
    done
  done
done
