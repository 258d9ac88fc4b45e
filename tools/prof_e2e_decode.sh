#!/bin/bash
# Config 5 decode through llama.cpp: the boundary's per-call phases (LAMM_HIP_STATS) and the kernels'
# own durations in that setting (rocprofv3 kernel trace), short context (-p 32 -n 64).
# usage (via gpurun): bash tools/prof_e2e_decode.sh gpurun_out/<dir> [threads]
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/e2e_decode}
T=${2:-16}
mkdir -p "$OUT"
M=$TMPDIR/lamm_synth_llama7b_q4_0.gguf
timeout -k 10 120 integration/_build/llama_e2e_hip -m "$M" --write-only > /dev/null 2>&1
LAMM_HIP_STATS=1 timeout -k 10 200 integration/_build/llama_e2e_hip -m "$M" -t $T -p 32 -n 64 > "$OUT/stats_t$T.json" 2> "$OUT/stats_t$T.err"
grep "lamm_hip stats" "$OUT/stats_t$T.err" > "$OUT/stats_t$T.txt" || true
rm -rf "$OUT/kt"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- integration/_build/llama_e2e_hip -m "$M" -t $T -p 32 -n 64 > "$OUT/kt_t$T.json" 2> "$OUT/kt_t$T.err"
find "$OUT/kt" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats_t$T.csv" \;
find "$OUT/kt" -name "*kernel_trace.csv" -exec cp {} "$OUT/kernel_trace_t$T.csv" \;
rm -rf "$OUT/kt"
