# Write-through (sc0 sc1) stores for short launches' results -- the flat GEMV's C, the fp6
# activation prep's planes, the K-group GEMM's C -- against tools/_old (the commit before):
# parity tests of those kernels, then the bench's config 2 + config 3 lines, 3 x alternating.
# Usage (via gpurun): bash tools/ab_write_through.sh OUT
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/ab_wt}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "row_slab or row_per_wave or gemv or golden or gemm or fp6 or config3 or config4" --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --no-llama --no-cpu --no-config1 --no-config4 > "$OUT/new_$i.json" 2>/dev/null
  LAMM_HIP_LIB=$PWD/tools/_old/liblamm_hip.so timeout -k 10 300 python -u bench.py --no-llama --no-cpu --no-config1 --no-config4 > "$OUT/old_$i.json" 2>/dev/null
done
