# dq16 ablations (loads only / compute only / NBUF 3 / clocks), one process per probe build
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/dq2}
mkdir -p "$OUT"
V=la-llama.cpp_amd/var_dq
for lib in la-llama.cpp_amd/liblamm_hip.so $V/liblamm_hip_dq_loads.so $V/liblamm_hip_dq_compute.so $V/liblamm_hip_dq_clock.so \
           $V/liblamm_hip_dq_nb3.so $V/liblamm_hip_dq_nb3loads.so $V/liblamm_hip_dq_nb3clock.so; do
  LAMM_HIP_LIB=$lib timeout -k 10 120 python -u tools/dq_ab.py q4_0 >> "$OUT/ab.jsonl" 2>> "$OUT/ab.err"
done
for lib in la-llama.cpp_amd/liblamm_hip.so $V/liblamm_hip_dq_loads.so $V/liblamm_hip_dq_compute.so $V/liblamm_hip_dq_clock.so; do
  LAMM_HIP_LIB=$lib timeout -k 10 120 python -u tools/dq_ab.py q4_0 4096 512 11008 >> "$OUT/ab.jsonl" 2>> "$OUT/ab.err"
done
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=40 --timeout 300 --timeout-method thread \
  --deselect "tests/test_benchmark_driver.py::test_llama_bench_sharded_decode_bitexact" > "$OUT/pytest_gpu.log" 2>&1 || [ $? -eq 1 ]
timeout -k 10 120 la-llama.cpp_amd/llama-matmul-bench -l 2 -i 2 --shard 8 -n 1 --dump "$OUT/g8.bin" > "$OUT/g8.log" 2>&1
