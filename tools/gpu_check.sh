# One GPU call: the GEMV and GEMM-stream probes, every -m gpu test (one process), then (3rd arg
# "bench") the default bench line -- each step under its own time limit; stops at the first failure.
# Usage (via gpurun): bash tools/gpu_check.sh gpurun_out/<dir> [tests|skip] [bench]
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/check}
mkdir -p "$OUT"
timeout -k 10 180 tools/gemv_probe > "$OUT/gemv_probe.json" 2> "$OUT/gemv_probe.err"
timeout -k 10 120 tools/gemm_stream_probe > "$OUT/gemm_stream_probe.json" 2> "$OUT/gemm_stream_probe.err"
if [ "${2:-tests}" = "tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
fi
if [ "$3" = "bench" ]; then
  timeout -k 10 900 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
fi
