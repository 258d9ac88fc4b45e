#!/bin/bash
# Config 5 through llama.cpp at several ggml pool widths: pp512, tg128 behind the prompt and
# llama-bench's own tg128 (from an empty cache), with the box's cgroup CPU quota and its
# throttling counters read around every run (is a 16-thread pool throttled on a 16-CPU share?).
# usage: tools/gpu_e2e_threads.sh [out_dir] [threads...]
OUT=${1:-gpurun_out/e2e_threads}
shift
THREADS=${@:-16 8 12 4}
mkdir -p "$OUT"
M=${TMPDIR:-/tmp}/lamm_synth_llama7b_q4_0.gguf
CG=/sys/fs/cgroup
{ echo "nproc $(nproc)"; cat $CG/cpu.max 2>/dev/null; cat /proc/self/status | grep -i cpus_allowed_list; } > "$OUT/cgroup.txt"
timeout -k 10 120 integration/_build/llama_e2e_hip -m "$M" --write-only 2>/dev/null || exit 1
for t in $THREADS; do
  cat $CG/cpu.stat > "$OUT/t$t.cpustat_before" 2>/dev/null
  LAMM_HIP_STATS=1 timeout -k 10 300 integration/_build/llama_e2e_hip -m "$M" -t $t -p 512 -n 128 > "$OUT/t$t.json" 2> "$OUT/t$t.err" || exit 1
  cat $CG/cpu.stat > "$OUT/t$t.cpustat_after" 2>/dev/null
  echo "t$t $(cat $OUT/t$t.json | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["pp_tok_s"], d["tg_tok_s"], d["tg_from_empty_tok_s"])')"
done
