# GPU step (via gpurun): llama.cpp pp512 + tg64 through the boundary in each float-order mode,
# with the boundary's own per-engine statistics, then the reference-order run under the kernel tracer.
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/modes}
mkdir -p "$OUT"
EXE=integration/_build/llama_e2e_hip
timeout -k 10 120 $EXE --write-only --regen > "$OUT/write.log" 2>&1
for mode in fast reference reference_views; do
  case $mode in
    fast) env_set="LAMM_HIP_ORDER=fast" ;;
    reference) env_set="LAMM_HIP_ORDER=reference" ;;
    reference_views) env_set="LAMM_HIP_ORDER=reference LAMM_HIP_VIEWS=1" ;;
  esac
  env $env_set LAMM_HIP_STATS=1 timeout -k 10 200 $EXE -t 16 -p 512 -n 64 > "$OUT/$mode.json" 2> "$OUT/$mode.err"
done
rm -rf "$OUT/prof"
LAMM_HIP_ORDER=reference timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- $EXE -t 16 -p 512 -n 64 > "$OUT/prof.json" 2> "$OUT/prof.err"
