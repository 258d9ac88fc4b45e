#!/bin/bash
# Config 5 end to end on the GPU box: llama.cpp-b2430 (unchanged) + liblamm_hip.so vs the
# reference's own lamm opt-3 AVX2 build, synthetic Llama-7B Q4_0 GGUF (32 blocks).
# usage: tools/e2e_llama.sh [out_dir]
set -o pipefail
OUT=${1:-gpurun_out/e2e}
mkdir -p "$OUT"
M=${TMPDIR:-/tmp}/lamm_synth_llama7b_q4_0.gguf
timeout -k 10 120 integration/_build/llama_e2e_hip -m "$M" --write-only 2> "$OUT/write.err" || exit 1
ls -la "$M" > "$OUT/model.txt"
for t in 1 4 16; do
  for views in 0 1; do
    echo "== hip t=$t LAMM_HIP_VIEWS=$views" >> "$OUT/hip.txt"
    LAMM_HIP_VIEWS=$views timeout -k 10 300 integration/_build/llama_e2e_hip -m "$M" -t $t -p 512 -n 128 \
      >> "$OUT/hip.txt" 2>> "$OUT/hip.err" || exit 1
  done
done
echo "== cpu reference lamm3 t=16" >> "$OUT/cpu.txt"
timeout -k 10 300 oracle/_ref/llama_e2e_lamm3 -m "$M" -t 16 -p 64 -n 16 >> "$OUT/cpu.txt" 2>> "$OUT/cpu.err" || exit 1
