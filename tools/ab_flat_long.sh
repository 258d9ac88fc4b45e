# A/B of the 6-run flat decode GEMV (and the q2_K row-per-wave GEMV: its parity tests, then the
# bench's config-4 line) (ffn_down's K = 11008) against the previous library
# (tools/_old/liblamm_hip.so, built from the commit before it): parity tests of the row-per-wave /
# flat kernels, then the device-API decode step 3 times each, alternating.
# Usage (via gpurun): bash tools/ab_flat_long.sh gpurun_out/<dir>
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/ab_flat_long}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "row_per_wave or multi_segment or q2k" --timeout 300 --timeout-method thread > "$OUT/pytest_rpw.log" 2>&1
B=la-llama.cpp_amd/llama-matmul-bench
for r in 1 2 3; do
  for args in "-n 1 --batch-proj" "-n 1"; do
    echo "new $args: $(timeout -k 10 120 $B $args -i 50 | tail -1)" >> "$OUT/ab.txt"
    echo "old $args: $(LD_LIBRARY_PATH=$PWD/tools/_old timeout -k 10 120 $B $args -i 50 | tail -1)" >> "$OUT/ab.txt"
  done
done
timeout -k 10 300 python -u bench.py --no-llama --no-cpu --no-config1 --no-gemm > "$OUT/bench_config4.json" 2> "$OUT/bench_config4.err"
