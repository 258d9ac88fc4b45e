#!/bin/bash
# boundary transfer modes (LAMM_HIP_ZERO_COPY) x activation modes, llama.cpp decode (p=32 n=64)
OUT=${1:-gpurun_out/ab_zc}
mkdir -p "$OUT"
M=${TMPDIR:-/tmp}/lamm_synth_llama7b_q4_0.gguf
timeout -k 10 120 integration/_build/llama_e2e_hip -m "$M" --write-only 2>/dev/null || exit 1
for zc in 0 in out both; do
  for fu in 1 0; do
    LAMM_HIP_ZERO_COPY=$zc LAMM_HIP_FUSED=$fu LAMM_HIP_STATS=1 timeout -k 10 300 integration/_build/llama_e2e_hip -m "$M" -t 8 -p 32 -n 64 > "$OUT/r.json" 2> "$OUT/r.err" || exit 1
    echo "zc=$zc fused=$fu $(python3 -c 'import json; d=json.load(open("'$OUT'/r.json")); print("tg %.2f tok/s" % d["tg_tok_s"])') $(grep 'N<=8' $OUT/r.err | head -1 | cut -c40-)" | tee -a "$OUT/ab.txt"
  done
done
