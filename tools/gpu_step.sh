# One GPU step of the round's work (via gpurun): the reference-order kernels' parity and timing,
# the k-quant GEMVs, the boundary and the 2-layer llama.cpp e2e, then the config-2 roofline.
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/g1}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_ref_order.py -x -q --timeout 120 --timeout-method thread > "$OUT/ref.log" 2>&1
timeout -k 10 200 python -u tools/ref_order_time.py > "$OUT/ref_time.log" 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "gemv_kq_row_per_wave" > "$OUT/kq.log" 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_ggml_boundary.py tests/test_gpu_reference_ggml.py -x -q --timeout 120 --timeout-method thread > "$OUT/bnd.log" 2>&1
timeout -k 10 900 python -u -m pytest tests/test_gpu_llama_e2e.py -x -v --timeout 300 --timeout-method thread -k "not 32_layers" > "$OUT/e2e2.log" 2>&1
bash tools/roofline_trace.sh "$OUT/rt" --no-cpu
