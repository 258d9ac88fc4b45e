# skinny N (2..8): GEMV kernels vs the prefill GEMM engines (LAMM_GEMV_MAX_N=1 routes N >= 2
# to the GEMMs), stationary weights, > MALL per launch; profiles/r01/gemv_vs_gemm_n.txt
set -e
echo "== GEMV (default)"
timeout -k 10 300 python3 -u tools/bench_gemv_n.py ${FMTS:-q4_0,q5_1,q8_0,q2_k,q4_k,q6_k,f16}
echo "== GEMM engines (LAMM_GEMV_MAX_N=1)"
LAMM_GEMV_MAX_N=1 timeout -k 10 300 python3 -u tools/bench_gemv_n.py ${FMTS:-q4_0,q5_1,q8_0,q2_k,q4_k,q6_k,f16}
