#!/bin/bash
# Config 5 decode through llama.cpp with ggml's pool left to the scheduler vs pinned (taskset) to
# 16 / 8 cores next to the GPU: does cross-socket / cross-CCD barrier traffic set the CPU side?
OUT=${1:-gpurun_out/e2e_pin}
mkdir -p "$OUT"
M=${TMPDIR:-/tmp}/lamm_synth_llama7b_q4_0.gguf
{ lscpu; for d in /sys/class/drm/card*/device; do echo "$d numa $(cat $d/numa_node 2>/dev/null) cpus $(cat $d/local_cpulist 2>/dev/null)"; done; } > "$OUT/topo.txt" 2>&1
LOCAL=$(python3 - <<'PY'
import glob
for d in sorted(glob.glob('/sys/class/drm/card*/device/local_cpulist')):
    s = open(d).read().strip()
    if s:
        cpus = []
        for part in s.split(','):
            a, _, b = part.partition('-')
            cpus += list(range(int(a), int(b or a) + 1))
        print(','.join(map(str, cpus[:16])))
        break
PY
)
echo "local $LOCAL" >> "$OUT/topo.txt"
[ -n "$LOCAL" ] || exit 1
timeout -k 10 120 integration/_build/llama_e2e_hip -m "$M" --write-only 2>/dev/null || exit 1
L8=$(echo $LOCAL | cut -d, -f1-8)
for rep in 0 1; do
  for cfg in "16 free" "16 pin" "8 free" "8 pin"; do
    set -- $cfg
    t=$1; mode=$2
    if [ $mode = pin ]; then CPUS=$LOCAL; [ $t = 8 ] && CPUS=$L8; PRE="taskset -c $CPUS"; else PRE=""; fi
    timeout -k 10 300 $PRE integration/_build/llama_e2e_hip -m "$M" -t $t -p 512 -n 128 > "$OUT/t${t}_${mode}_$rep.json" 2> "$OUT/t${t}_${mode}_$rep.err" || exit 1
    echo "t$t $mode $rep $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["pp_tok_s"], d["tg_tok_s"], d["tg_from_empty_tok_s"])' $OUT/t${t}_${mode}_$rep.json)" | tee -a "$OUT/summary.txt"
  done
done
