#!/bin/bash
# Config 5 through llama.cpp with each LAMM_HIP_POOL mode (0: thread 0 alone; 1: the pool quantizes
# the prefill activations, the default; 3: and scatters C out of pinned memory), alternating.
OUT=${1:-gpurun_out/e2e_pool_modes}
mkdir -p "$OUT"
M=${TMPDIR:-/tmp}/lamm_synth_llama7b_q4_0.gguf
timeout -k 10 120 integration/_build/llama_e2e_hip -m "$M" --write-only 2>/dev/null || exit 1
for rep in 0 1; do
  for pool in ${POOLS:-1 3 0}; do
    tag=pool${pool}_$rep
    LAMM_HIP_POOL=$pool timeout -k 10 300 integration/_build/llama_e2e_hip -m "$M" -t 16 -p 512 -n 128 > "$OUT/$tag.json" 2> "$OUT/$tag.err" || exit 1
    echo "$tag $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["pp_tok_s"], d["tg_tok_s"], d["tg_from_empty_tok_s"])' $OUT/$tag.json)" | tee -a "$OUT/summary.txt"
  done
done
