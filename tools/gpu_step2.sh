# GPU step (via gpurun): reference-order parity (incl. the MFMA prefill form) and timing, config-2
# roofline measurements, then the 32-layer llama.cpp parity tests.
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/g3}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_ref_order.py -x -q --timeout 120 --timeout-method thread > "$OUT/ref.log" 2>&1
timeout -k 10 200 python -u tools/ref_order_time.py > "$OUT/ref_time.log" 2>&1
bash tools/roofline_trace.sh "$OUT/rt" --no-cpu
timeout -k 10 1000 python -u -m pytest tests/test_gpu_llama_e2e.py -x -v -s --timeout 400 --timeout-method thread -k "32_layers" > "$OUT/e2e32.log" 2>&1
