# Kernel statistics of the device-API decode step (llama-matmul-bench, batched projections, with and
# without the attention matmuls) and the new attention self-check test.
# Usage (via gpurun): bash tools/prof_decode_step.sh gpurun_out/<dir>
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/decode_prof}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_benchmark_driver.py -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/pytest_bench_driver.log" 2>&1
B=la-llama.cpp_amd/llama-matmul-bench
rm -rf "$OUT/p1" "$OUT/p2"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/p1" -o run -- $B -n 1 --batch-proj -i 20 > "$OUT/step.txt" 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/p2" -o run -- $B -n 1 --batch-proj --ctx 512 -i 20 > "$OUT/step_ctx512.txt" 2>&1
