# dq16 v2 with / without the L2 prefetch phase, the dq16 parity tests, the 8-rank sharded run
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/dq4}
mkdir -p "$OUT"
V=la-llama.cpp_amd/var_dq
for shape in "4096 512 4096" "4096 512 11008"; do
for lib in la-llama.cpp_amd/liblamm_hip.so $V/liblamm_hip_dq_v2nopf.so $V/liblamm_hip_dq_v2pfnbv2.so $V/liblamm_hip_dq_v3.so $V/liblamm_hip_dq_v3nopf.so; do
  LAMM_HIP_LIB=$lib timeout -k 10 120 python -u tools/dq_ab.py q4_0 $shape >> "$OUT/ab.jsonl" 2>> "$OUT/ab.err"
done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "dq16 or config3" --timeout 300 --timeout-method thread > "$OUT/pytest_dq.log" 2>&1 || [ $? -eq 1 ]
timeout -k 10 120 la-llama.cpp_amd/llama-matmul-bench -l 2 -i 2 --shard 8 -n 1 --dump "$OUT/g8.bin" > "$OUT/g8.log" 2>&1
timeout -k 10 300 python -u -m pytest tests/test_benchmark_driver.py -m gpu -q --timeout 300 --timeout-method thread > "$OUT/pytest_driver.log" 2>&1
