#!/bin/bash
# Config 5 through llama.cpp: prefill pool jobs (LAMM_HIP_POOL=1) with the helpers spinning until
# thread 0 finishes (LAMM_HIP_HELPERS=0) vs asleep on a futex once their job is done (=3), and
# thread 0 alone (LAMM_HIP_POOL=0) -- do spinning pool threads slow the call's PCIe transfers?
OUT=${1:-gpurun_out/e2e_pool_sleep}
mkdir -p "$OUT"
M=${TMPDIR:-/tmp}/lamm_synth_llama7b_q4_0.gguf
timeout -k 10 120 integration/_build/llama_e2e_hip -m "$M" --write-only 2>/dev/null || exit 1
for rep in 0 1; do
  for cfg in "1 0" "1 3" "0 0" "0 3"; do
    set -- $cfg
    tag=pool$1_h$2_$rep
    LAMM_HIP_POOL=$1 LAMM_HIP_HELPERS=$2 LAMM_HIP_STATS=1 timeout -k 10 300 integration/_build/llama_e2e_hip -m "$M" -t 16 -p 512 -n 128 > "$OUT/$tag.json" 2> "$OUT/$tag.err" || exit 1
    echo "$tag $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["pp_tok_s"], d["tg_tok_s"], d["tg_from_empty_tok_s"])' $OUT/$tag.json) | $(grep 'weights N>8' $OUT/$tag.err | sed 's/.*us\/call//')" | tee -a "$OUT/summary.txt"
  done
done
