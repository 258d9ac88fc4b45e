# dq16 v2 PMC passes (where the waves' cycles go), its parity tests, the 8-rank sharded run
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/dq5}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "dq16 or config3" --timeout 300 --timeout-method thread > "$OUT/pytest_dq.log" 2>&1 || [ $? -eq 1 ]
timeout -k 10 120 la-llama.cpp_amd/llama-matmul-bench -l 2 -i 2 --shard 8 -n 1 --dump "$OUT/g8.bin" > "$OUT/g8.log" 2>&1 || true
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_BUSY_CYCLES --output-format csv -d "$OUT/pmc1" -o run -- python3 tools/dq_ab.py q4_0 > "$OUT/pmc1.log" 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU SQ_ACTIVE_INST_MISC --output-format csv -d "$OUT/pmc2" -o run -- python3 tools/dq_ab.py q4_0 > "$OUT/pmc2.log" 2>&1
timeout -k 10 300 python -u -m pytest tests/test_benchmark_driver.py -m gpu -q --timeout 300 --timeout-method thread > "$OUT/pytest_driver.log" 2>&1
