# The looping flat GEMV (LAMM_GEMV_LOOP = workgroups; 0 = one row group per workgroup): its parity
# tests, single q4_0 calls at the Llama-7B projection sizes, and the device-API decode step
# (separate and batched projections, F32 activations) 3 x alternating over the grid sizes.
# Usage (via gpurun): bash tools/ab_gemv_loop.sh gpurun_out/<dir>
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/ab_gemv_loop}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "flat_loop or row_slab or row_per_wave" --timeout 300 --timeout-method thread > "$OUT/pytest_loop.log" 2>&1
for L in 0 512 1024 2048; do
  for mk in "12288 4096" "22016 4096" "11008 4096"; do
    set -- $mk
    echo "loop=$L $(LAMM_GEMV_LOOP=$L timeout -k 10 120 python -u tools/bench_gemv_n.py q4_0 $1 $2)" >> "$OUT/single.txt"
  done
done
B=la-llama.cpp_amd/llama-matmul-bench
for r in 1 2 3; do
  for L in 0 512 1024 2048; do
    for args in "-n 1 --batch-proj" "-n 1"; do
      echo "loop=$L $args: $(LAMM_GEMV_LOOP=$L timeout -k 10 120 $B $args -i 50 | tail -1)" >> "$OUT/step.txt"
    done
  done
done
