# GPU step (via gpurun): reference-order parity tests, kernel times (tools/ref_ab.py) and the SQ
# counters of the prefill GEMM / F16 kernel
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/ab}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_ref_order.py -x -q --timeout 120 --timeout-method thread > "$OUT/ref.log" 2>&1
timeout -k 10 200 python3 -u tools/ref_ab.py > "$OUT/default.json" 2> "$OUT/default.err"
bash tools/gpu_pmc_ref.sh "$OUT/pmc"
