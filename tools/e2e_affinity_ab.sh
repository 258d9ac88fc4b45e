#!/bin/bash
# Decode through llama.cpp with the process pinned to a CPU list (taskset) and ggml's threads kept
# inside it (--numa numactl), against the unpinned run, alternating; -p 32 -n 64.
# usage (via gpurun): bash tools/e2e_affinity_ab.sh gpurun_out/<dir> REPS "T:CPULIST" ...  (CPULIST "-": unpinned)
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/e2e_affinity}
REPS=${2:-3}
shift 2
mkdir -p "$OUT"
M=$TMPDIR/lamm_synth_llama7b_q4_0.gguf
timeout -k 10 120 integration/_build/llama_e2e_hip -m "$M" --write-only > /dev/null 2>&1
for r in $(seq 1 $REPS); do
  for s in "$@"; do
    t=${s%%:*}; cpus=${s#*:}
    name="t${t}_${cpus//[,-]/_}"
    if [ "$cpus" = "-" ]; then
      timeout -k 10 200 integration/_build/llama_e2e_hip -m "$M" -t $t -p 32 -n 64 > "$OUT/${name}_r$r.json" 2>/dev/null
    else
      timeout -k 10 200 taskset -c "$cpus" integration/_build/llama_e2e_hip -m "$M" -t $t --numa numactl -p 32 -n 64 > "$OUT/${name}_r$r.json" 2>/dev/null
    fi
    echo "$name r=$r $(grep -o '"tg_from_empty_tok_s": [0-9.]*' "$OUT/${name}_r$r.json")" >> "$OUT/summary.txt"
  done
done
