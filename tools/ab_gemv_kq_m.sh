# The row-per-wave k-quant GEMV against the wave-group kernels at larger M (11008 = ffn rows,
# 32000 = output.weight rows), K = 4096.  Usage (via gpurun): bash tools/ab_gemv_kq_m.sh gpurun_out/<dir>
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/ab_kq_m}
mkdir -p "$OUT"
for M in 11008 32000; do
  timeout -k 10 250 python -u tools/bench_gemv_n.py q2_k,q4_k,q5_k $M 4096 > "$OUT/rpw_M$M.json" 2> "$OUT/rpw_M$M.err"
  LAMM_GEMV_RPW=0 timeout -k 10 250 python -u tools/bench_gemv_n.py q2_k,q4_k,q5_k $M 4096 > "$OUT/wg_M$M.json" 2> "$OUT/wg_M$M.err"
done
