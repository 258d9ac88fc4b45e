#!/bin/bash
# llama.cpp decode through the boundary (p=32 n=64, -t 8): completion flag written by the GEMV's
# last workgroup (LAMM_HIP_KERNEL_SIGNAL=1) vs a separate signal launch (=0, the default), interleaved
OUT=${1:-gpurun_out/ab_ks}
mkdir -p "$OUT"
M=${TMPDIR:-/tmp}/lamm_synth_llama7b_q4_0.gguf
timeout -k 10 120 integration/_build/llama_e2e_hip -m "$M" --write-only 2>/dev/null || exit 1
for rep in 1 2; do
  for ks in 1 0; do
    LAMM_HIP_KERNEL_SIGNAL=$ks LAMM_HIP_STATS=1 timeout -k 10 300 integration/_build/llama_e2e_hip -m "$M" -t 8 -p 32 -n 64 > "$OUT/r.json" 2> "$OUT/r.err" || exit 1
    echo "kernel_signal=$ks $(python3 -c 'import json; d=json.load(open("'$OUT'/r.json")); print("tg %.2f tok/s" % d["tg_tok_s"])') $(grep 'N<=8' $OUT/r.err | head -1 | cut -c40-)" | tee -a "$OUT/ab.txt"
  done
done
