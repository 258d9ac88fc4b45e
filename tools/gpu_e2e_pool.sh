#!/bin/bash
# Config 5 prefill through llama.cpp with ggml's pool threads quantizing the activations (LAMM_HIP_POOL=1, the default)
# vs thread 0 alone (=0), alternating, with LAMM_HIP_STATS phases.
OUT=${1:-gpurun_out/e2e_pool}
THREADS=${2:-16}
mkdir -p "$OUT"
M=${TMPDIR:-/tmp}/lamm_synth_llama7b_q4_0.gguf
timeout -k 10 120 integration/_build/llama_e2e_hip -m "$M" --write-only 2>/dev/null || exit 1
for rep in 0 1; do
  for pool in 1 0; do
    LAMM_HIP_POOL=$pool LAMM_HIP_STATS=1 timeout -k 10 300 integration/_build/llama_e2e_hip -m "$M" -t $THREADS -p 512 -n 128 > "$OUT/pool${pool}_t${THREADS}_$rep.json" 2> "$OUT/pool${pool}_t${THREADS}_$rep.err" || exit 1
    echo "pool $pool t$THREADS rep $rep $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["pp_tok_s"], d["tg_tok_s"], d["tg_from_empty_tok_s"])' $OUT/pool${pool}_t${THREADS}_$rep.json)" | tee -a "$OUT/summary.txt"
  done
done
