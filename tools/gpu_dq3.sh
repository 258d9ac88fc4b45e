# dq16 v2 (coalesced, LDS-staged) ablations + the GPU suite + the 8-rank sharded run (call stack)
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/dq3}
mkdir -p "$OUT"
V=la-llama.cpp_amd/var_dq
for shape in "4096 512 4096" "4096 512 11008"; do
for lib in la-llama.cpp_amd/liblamm_hip.so $V/liblamm_hip_dq_v2loads.so $V/liblamm_hip_dq_v2clock.so \
           $V/liblamm_hip_dq_v2nbv2.so $V/liblamm_hip_dq_v2nbv2clock.so; do
  LAMM_HIP_LIB=$lib timeout -k 10 120 python -u tools/dq_ab.py q4_0 $shape >> "$OUT/ab.jsonl" 2>> "$OUT/ab.err"
done
done
timeout -k 10 300 python -u tools/dq_probe.py "$OUT/dq_probe.json" > "$OUT/dq_probe.log" 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=40 --timeout 300 --timeout-method thread \
  --deselect "tests/test_benchmark_driver.py::test_llama_bench_sharded_decode_bitexact" > "$OUT/pytest_gpu.log" 2>&1 || [ $? -eq 1 ]
timeout -k 10 120 la-llama.cpp_amd/llama-matmul-bench -l 2 -i 2 --shard 8 -n 1 --dump "$OUT/g8.bin" > "$OUT/g8.log" 2>&1
