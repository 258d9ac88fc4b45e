# decode-step GEMV launch variants on the Llama-7B weight-matmul step (one matrix per call)
set -e
B=./la-llama.cpp_amd/llama-matmul-bench
for v in 0 8 12 10; do
  echo "== LAMM_GEMV_VARIANT=$v"
  LAMM_GEMV_VARIANT=$v timeout -k 10 120 $B -d q4_0 -n 1 -i 50 | grep step
done
