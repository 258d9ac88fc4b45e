# Guarded staging loads (only the waves holding an activation block issue them) in the whole
# decode step: the GEMV parity tests, then llama-matmul-bench -n 1 (batched / separate projections)
# with this library vs tools/_old (the commit before), 3 x alternating, and the F32 / q8 single calls.
# Usage (via gpurun): bash tools/ab_stage_guard_step.sh OUT
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/ab_stage_guard_step}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "row_slab or row_per_wave or gemv or golden" --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
B=la-llama.cpp_amd/llama-matmul-bench
for r in 1 2 3; do
  for args in "-n 1 --batch-proj" "-n 1"; do
    echo "new $args: $(timeout -k 10 120 $B $args -i 50 | tail -1)" >> "$OUT/ab.txt"
    echo "old $args: $(LD_LIBRARY_PATH=$PWD/tools/_old timeout -k 10 120 $B $args -i 50 | tail -1)" >> "$OUT/ab.txt"
  done
done
timeout -k 10 200 python -u tools/gemv_f32_vs_q8.py > "$OUT/f32_vs_q8_new.json" 2>/dev/null
timeout -k 10 60 tools/gemv_probe lib > "$OUT/lib.json" 2>/dev/null
timeout -k 10 300 python -u bench.py --no-llama --no-cpu --no-config1 --no-gemm > "$OUT/bench_c2c4.json" 2> "$OUT/bench_c2c4.err"
