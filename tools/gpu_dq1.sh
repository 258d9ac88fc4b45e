# dq16 probe, the GPU suite (up to 40 failures listed), then the 8-rank sharded-decode run alone
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/dq1}
mkdir -p "$OUT"
timeout -k 10 300 python -u tools/dq_probe.py "$OUT/dq_probe.json" > "$OUT/dq_probe.log" 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=40 --timeout 300 --timeout-method thread \
  --deselect "tests/test_benchmark_driver.py::test_llama_bench_sharded_decode_bitexact" > "$OUT/pytest_gpu.log" 2>&1 || true
timeout -k 10 120 la-llama.cpp_amd/llama-matmul-bench -l 2 -i 2 --shard 8 -n 1 --dump "$OUT/g8.bin" > "$OUT/g8.log" 2>&1
