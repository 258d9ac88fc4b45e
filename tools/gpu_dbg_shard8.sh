# GPU suite minus the 8-rank sharded-decode test, then that run alone with its call stack on a fault
set -e
OUT=${1:-gpurun_out/dbg8}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  --deselect "tests/test_benchmark_driver.py::test_llama_bench_sharded_decode_bitexact" > "$OUT/pytest_gpu.log" 2>&1
timeout -k 10 120 la-llama.cpp_amd/llama-matmul-bench -l 2 -i 2 --shard 8 -n 1 --dump "$OUT/g8.bin" > "$OUT/g8.log" 2>&1
