# Write-through plane stores in the F32-activation fp6 prep (prefill with ggml's F32 src1) against
# tools/_old (the commit before): GEMM parity tests, then llama-matmul-bench -n 512 (prefill, F32
# activations) 3 x alternating.  Usage (via gpurun): bash tools/ab_prep_f32_wt.sh OUT
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/ab_prep_f32_wt}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_quantize.py -m gpu -x -q -k "gemm or fp6 or f32 or config3" --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
B=la-llama.cpp_amd/llama-matmul-bench
for r in 1 2 3; do
  echo "new: $(timeout -k 10 120 $B -n 512 -i 10 | tail -1)" >> "$OUT/ab.txt"
  echo "old: $(LD_LIBRARY_PATH=$PWD/tools/_old timeout -k 10 120 $B -n 512 -i 10 | tail -1)" >> "$OUT/ab.txt"
done
