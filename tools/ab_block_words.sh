# Weight blocks loaded as ceil((BPB + 2) / 4) dwords instead of (BPB + 3) / 4 + 1 (row-per-wave and
# flat GEMVs) against tools/_old (the commit before): GEMV parity tests, then config 2 through the
# library (probe "lib") 4 x alternating, the bench's config 2 + config 4 lines 2 x alternating and
# the decode step 2 x alternating.  Usage (via gpurun): bash tools/ab_block_words.sh OUT
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/ab_block_words}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "row_slab or row_per_wave or gemv or golden" --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
for i in 1 2 3 4; do
  echo "new $(timeout -k 10 60 tools/gemv_probe lib 2>/dev/null)" >> "$OUT/probe.txt"
  echo "old $(LD_LIBRARY_PATH=$PWD/tools/_old timeout -k 10 60 tools/gemv_probe lib 2>/dev/null)" >> "$OUT/probe.txt"
done
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-llama --no-cpu --no-config1 --no-gemm > "$OUT/new_$i.json" 2>/dev/null
  LAMM_HIP_LIB=$PWD/tools/_old/liblamm_hip.so timeout -k 10 300 python -u bench.py --no-llama --no-cpu --no-config1 --no-gemm > "$OUT/old_$i.json" 2>/dev/null
done
B=la-llama.cpp_amd/llama-matmul-bench
for r in 1 2; do
  for args in "-n 1 --batch-proj" "-n 1"; do
    echo "new $args: $(timeout -k 10 120 $B $args -i 50 | tail -1)" >> "$OUT/step.txt"
    echo "old $args: $(LD_LIBRARY_PATH=$PWD/tools/_old timeout -k 10 120 $B $args -i 50 | tail -1)" >> "$OUT/step.txt"
  done
done
