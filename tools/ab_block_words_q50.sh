# q5_0 keeps its 7-dword block loads (block_dwords): GEMV parity, then the bench's config 4 GEMV
# lines against tools/_old 2 x alternating.  Usage (via gpurun): bash tools/ab_block_words_q50.sh OUT
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/ab_block_words_q50}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "row_slab or row_per_wave or gemv or golden" --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-llama --no-cpu --no-config1 --no-gemm > "$OUT/new_$i.json" 2>/dev/null
  LAMM_HIP_LIB=$PWD/tools/_old/liblamm_hip.so timeout -k 10 300 python -u bench.py --no-llama --no-cpu --no-config1 --no-gemm > "$OUT/old_$i.json" 2>/dev/null
done
