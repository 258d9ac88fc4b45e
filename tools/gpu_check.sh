# One GPU call: the GEMV and GEMM-stream probes, then every -m gpu test (one process) -- each
# step under its own time limit; stops at the first failure.
# Usage (via gpurun): bash tools/gpu_check.sh gpurun_out/<dir> [skip-tests]
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/check}
mkdir -p "$OUT"
timeout -k 10 180 tools/gemv_probe > "$OUT/gemv_probe.json" 2> "$OUT/gemv_probe.err"
timeout -k 10 120 tools/gemm_stream_probe > "$OUT/gemm_stream_probe.json" 2> "$OUT/gemm_stream_probe.err"
if [ -z "$2" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
fi
