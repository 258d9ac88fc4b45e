# One GPU call for the ggml boundary's transfer costs: the host<->device copy probe, the
# reference's ggml + liblamm_hip.so on the config-5 prefill shapes with per-phase LAMM_HIP_STATS,
# llama.cpp end to end with stats (tools/e2e_stats.sh), the device-API decode step with and
# without the attention matmuls (--ctx), and (2nd arg "tests") every -m gpu test first.
# Usage (via gpurun): bash tools/gpu_boundary_probe.sh gpurun_out/<dir> [tests]
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/bnd}
mkdir -p "$OUT"
if [ "$2" = "tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
fi
timeout -k 10 120 tools/xfer_probe > "$OUT/xfer_probe.json" 2> "$OUT/xfer_probe.err"
for nth in 1 8 16; do
  for shape in "4096 512 4096" "11008 512 4096"; do
    set -- $shape
    echo "== q4_0 M=$1 N=$2 K=$3 threads=$nth" >> "$OUT/ref_driver_stats.txt"
    LAMM_HIP_STATS=1 timeout -k 10 120 oracle/_ref/ref_driver_hip bench q4_0 $1 $2 $3 $nth 20 5 >> "$OUT/ref_driver_stats.txt" 2>&1
  done
done
B=la-llama.cpp_amd/llama-matmul-bench
timeout -k 10 120 $B -n 1 --batch-proj > "$OUT/step_decode.txt" 2>&1
timeout -k 10 120 $B -n 1 --batch-proj --ctx 512 > "$OUT/step_decode_ctx512.txt" 2>&1
timeout -k 10 120 $B -n 1 --ctx 512 > "$OUT/step_decode_ctx512_sep.txt" 2>&1
bash tools/e2e_stats.sh "$OUT/stats" 8 16
