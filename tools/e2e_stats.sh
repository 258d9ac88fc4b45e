#!/bin/bash
# decode/prefill split of a llama.cpp token between the boundary (LAMM_HIP_STATS) and the rest
# usage: tools/e2e_stats.sh [out_dir] [threads...]   (default threads: 16)
OUT=${1:-gpurun_out/stats}
shift
THREADS=${@:-16}
mkdir -p "$OUT"
M=${TMPDIR:-/tmp}/lamm_synth_llama7b_q4_0.gguf
timeout -k 10 120 integration/_build/llama_e2e_hip -m "$M" --write-only 2>/dev/null || exit 1
for t in $THREADS; do
  for p in 32 512; do
    LAMM_HIP_STATS=1 timeout -k 10 300 integration/_build/llama_e2e_hip -m "$M" -t $t -p $p -n 64 > "$OUT/p${p}_t$t.json" 2> "$OUT/p${p}_t$t.err" || exit 1
    grep "lamm_hip stats" "$OUT/p${p}_t$t.err" > "$OUT/p${p}_t$t.stats"
  done
done
