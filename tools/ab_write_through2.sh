# Write-through C tiles in the whole-tile fp6 GEMM, the i8 GEMM and the k-quant GEMM (CTile)
# against tools/_old (the commit before): their parity tests, then the bench's config 3 + config 4
# lines, 3 x alternating.  Usage (via gpurun): bash tools/ab_write_through2.sh OUT
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/ab_wt2}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "gemm or fp6 or config3 or config4 or golden or split" --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --no-llama --no-cpu --no-config1 > "$OUT/new_$i.json" 2>/dev/null
  LAMM_HIP_LIB=$PWD/tools/_old/liblamm_hip.so timeout -k 10 300 python -u bench.py --no-llama --no-cpu --no-config1 > "$OUT/old_$i.json" 2>/dev/null
done
