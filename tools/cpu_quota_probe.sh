#!/bin/bash
# CPU-quota evidence for the decode thread scaling: the box's cgroup CPU limit and its
# throttling counters around one llama.cpp decode run per thread count.
# usage (via gpurun): bash tools/cpu_quota_probe.sh gpurun_out/<dir> THREADS...
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/cpu_quota}
shift
mkdir -p "$OUT"
M=$TMPDIR/lamm_synth_llama7b_q4_0.gguf
timeout -k 10 120 integration/_build/llama_e2e_hip -m "$M" --write-only > /dev/null 2>&1
{
  echo "nproc $(nproc)"
  echo "cpu.max $(cat /sys/fs/cgroup/cpu.max 2>/dev/null || echo n/a)"
  echo "cpuset $(cat /sys/fs/cgroup/cpuset.cpus.effective 2>/dev/null || echo n/a)"
  echo "affinity $(python3 -c 'import os; print(len(os.sched_getaffinity(0)))')"
} > "$OUT/summary.txt"
for t in "$@"; do
  before=$(cat /sys/fs/cgroup/cpu.stat 2>/dev/null | tr '\n' ' ')
  timeout -k 10 200 integration/_build/llama_e2e_hip -m "$M" -t $t -p 32 -n 64 > "$OUT/t$t.json" 2> "$OUT/t$t.err"
  after=$(cat /sys/fs/cgroup/cpu.stat 2>/dev/null | tr '\n' ' ')
  echo "t=$t $(grep -o '"tg_tok_s": [0-9.]*' "$OUT/t$t.json") before: $before after: $after" >> "$OUT/summary.txt"
done
