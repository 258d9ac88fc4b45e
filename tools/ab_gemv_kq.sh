# The row-per-wave k-quant decode GEMVs (q2_K / q4_K / q5_K): their parity tests, then single-call
# timing per format with them (default) and without (LAMM_GEMV_RPW=0: the wave-group kernels).
# Usage (via gpurun): bash tools/ab_gemv_kq.sh gpurun_out/<dir>
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/ab_kq}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "kq_row_per_wave or multi_segment or golden" --timeout 300 --timeout-method thread > "$OUT/pytest_kq.log" 2>&1
timeout -k 10 250 python -u tools/bench_gemv_n.py q4_0,q2_k,q4_k,q5_k,q6_k,f16 > "$OUT/gemv_formats.json" 2> "$OUT/gemv_formats.err"
LAMM_GEMV_RPW=0 timeout -k 10 250 python -u tools/bench_gemv_n.py q4_0,q2_k,q4_k,q5_k > "$OUT/gemv_formats_rpw0.json" 2> "$OUT/gemv_formats_rpw0.err"
