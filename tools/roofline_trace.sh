#!/bin/bash
# Config 2's kernel, measured several ways on one box (via gpurun):
#   1. bench.py as the driver runs it (--steps 20 --warmup 5), its roofline from isolated launches
#   2. the same bench.py command under rocprofv3 --kernel-trace --stats (the committed summary)
#   3. rocprofv3 --kernel-trace of tools/roofline_trace.py (host-paced launches; --sync-each: idle)
#   4. two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) of tools/pmc_flat1.py -> HBM bytes per launch
# Usage: bash tools/roofline_trace.sh gpurun_out/<dir> [extra bench args]
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/roofline}
shift || true
mkdir -p "$OUT"
rm -rf "$OUT/kt" "$OUT/kt_idle" "$OUT/pmc_f" "$OUT/pmc_w" "$OUT/bench_prof"
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 "$@" > "$OUT/bench.json" 2> "$OUT/bench.err"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/bench_prof" -o run -- python3 -u bench.py --steps 20 --warmup 5 "$@" > "$OUT/bench_under_rocprof.json" 2> "$OUT/bench_under_rocprof.err"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- python3 -u tools/roofline_trace.py > "$OUT/trace.log" 2>&1
python3 tools/kt_roofline.py "$(find "$OUT/kt" -name '*kernel_trace.csv' | head -1)" "$OUT/roofline_q4_0_gemv_single.json"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt_idle" -o run -- python3 -u tools/roofline_trace.py --sync-each --gap-us 20 > "$OUT/trace_idle.log" 2>&1
python3 tools/kt_roofline.py "$(find "$OUT/kt_idle" -name '*kernel_trace.csv' | head -1)" "$OUT/roofline_idle.json"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_f" -o f -- python3 tools/pmc_flat1.py > "$OUT/pmc_f.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_w" -o w -- python3 tools/pmc_flat1.py > "$OUT/pmc_w.log" 2>&1
python3 tools/pmc_traffic_flat1.py "$(find "$OUT/pmc_f" -name '*counter_collection.csv' | head -1)" \
  "$(find "$OUT/pmc_w" -name '*counter_collection.csv' | head -1)" "$OUT/traffic_q4_0_gemv_single.json"
