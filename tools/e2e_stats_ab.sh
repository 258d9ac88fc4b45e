#!/bin/bash
# Decode through llama.cpp with alternating settings: LAMM_HIP_STATS per-call phases + tok/s,
# -p 32 -n 64, -t 16 (T=<threads> in a setting changes it; NUMA=<strategy> passes --numa).  Each setting is
# NAME:VAR=VALUE[,VAR=VALUE] ("base:" for none).
# usage (via gpurun): bash tools/e2e_stats_ab.sh gpurun_out/<dir> REPS SETTING...
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/e2e_stats_ab}
REPS=${2:-2}
shift 2
mkdir -p "$OUT"
M=$TMPDIR/lamm_synth_llama7b_q4_0.gguf
timeout -k 10 120 integration/_build/llama_e2e_hip -m "$M" --write-only > /dev/null 2>&1
for r in $(seq 1 $REPS); do
  for s in "$@"; do
    name=${s%%:*}
    vars=${s#*:}
    envs=()
    IFS=',' read -ra kv <<< "$vars"
    t=16
    extra=()
    for x in "${kv[@]}"; do
      case "$x" in T=*) t=${x#T=} ;; NUMA=*) extra+=(--numa "${x#NUMA=}") ;; ?*) envs+=("$x") ;; esac
    done
    env "${envs[@]}" LAMM_HIP_STATS=1 timeout -k 10 200 integration/_build/llama_e2e_hip -m "$M" -t $t "${extra[@]}" -p 32 -n 64 > "$OUT/${name}_r$r.json" 2> "$OUT/${name}_r$r.err"
    echo "$name r=$r $(grep -o '"tg_tok_s": [0-9.]*' "$OUT/${name}_r$r.json") $(grep 'weights N<=8' "$OUT/${name}_r$r.err")" >> "$OUT/summary.txt"
  done
done
