# non-temporal C stores in the i8 (gemm3_kernel) and super-block (gemm_kq_kernel) GEMM epilogues:
# (run before they became the default) VAR = build_var/liblamm_hip_gnt.so (built from a copy of
# the sources with those stores NT) vs
# the default build.  Parity of the variant on the i8 / super-block tests, then REPS alternating
# process pairs of tools/ab_gemm_store.py.
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/gemm_store}
REPS=${REPS:-3}
VAR=la-llama.cpp_amd/build_var/liblamm_hip_gnt.so
mkdir -p "$OUT"
LAMM_HIP_LIB=$PWD/$VAR timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -k "i8 or q8_0 or q5_1 or q6_k or q4_k or q5_k or q2_k" > "$OUT/pytest_var.log" 2>&1
for rep in $(seq 1 $REPS); do
  timeout -k 10 200 python -u tools/ab_gemm_store.py > "$OUT/default_$rep.log" 2>&1
  LAMM_HIP_LIB=$PWD/$VAR timeout -k 10 200 python -u tools/ab_gemm_store.py > "$OUT/gnt_$rep.log" 2>&1
done
