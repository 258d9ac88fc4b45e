# Staging loads issued only by the waves that hold an activation block (flat / row-per-wave GEMV):
# the GEMV parity tests, then config 2 through the library (probe "lib", 3 runs) against the probe's
# G8 clone, and the bench's config-2 line.  Usage (via gpurun): bash tools/ab_stage_guard.sh OUT
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/ab_stage_guard}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "row_slab or row_per_wave or gemv or golden" --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
for i in 1 2 3; do
  timeout -k 10 100 tools/gemv_probe G8 > "$OUT/g8_$i.json" 2>/dev/null
  timeout -k 10 60 tools/gemv_probe lib > "$OUT/lib_$i.json" 2>/dev/null
done
timeout -k 10 300 python -u bench.py --no-llama --no-cpu --no-config1 --no-config4 --no-gemm > "$OUT/bench.json" 2> "$OUT/bench.err"
