# decode-step GEMV launch geometry on the Llama-7B weight-matmul step (one matrix per call):
# LAMM_GEMV_VARIANT 0 = 8 waves x 2 LDS slots per workgroup, 14 = 4 waves, 15 = 2 waves
set -e
B=./la-llama.cpp_amd/llama-matmul-bench
for v in 0 14 15 0; do
  echo "== LAMM_GEMV_VARIANT=$v"
  LAMM_GEMV_VARIANT=$v timeout -k 10 120 $B -d q4_0 -n 1 -i 50 | grep step
  LAMM_GEMV_VARIANT=$v timeout -k 10 120 $B -d q4_0 -n 1 -i 50 --batch-proj | grep step
done
