# GPU step (via gpurun): reference-order kernels (one-column producer/chain GEMV, F16 attention),
# the llama.cpp node / 32-layer parity tests, then the float-order modes end to end.
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/g4}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_ref_order.py tests/test_gpu_parity.py -k "ref or gemv"  -x -q --timeout 120 --timeout-method thread > "$OUT/ref.log" 2>&1
timeout -k 10 900 python -u -m pytest tests/test_gpu_llama_e2e.py -x -v -s --timeout 400 --timeout-method thread -k "nodes or 32_layers" > "$OUT/e2e.log" 2>&1
bash tools/gpu_e2e_modes.sh "$OUT/modes"
rm -rf "$OUT/rt_prof"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rt_prof" -o run -- python3 -u tools/ref_order_time.py > "$OUT/ref_time.log" 2>&1
