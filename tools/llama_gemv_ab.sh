# decode-step GEMV launch A/B on the Llama-7B weight-matmul step (one matrix per call).
# The record in profiles/r01/llama_decode_gemv_geometry_ab.txt compared LAMM_GEMV_VARIANT 0
# (8 waves x 2 LDS slots per workgroup) with two temporary builds (14: 4 waves, 15: 2 waves);
# those variants were not kept (+-2 %).  Today this runs the kept launch choices: 0 (default)
# and 10 (the VGPR-landing stream kernel).
set -e
B=./la-llama.cpp_amd/llama-matmul-bench
for v in 0 10; do
  echo "== LAMM_GEMV_VARIANT=$v"
  LAMM_GEMV_VARIANT=$v timeout -k 10 120 $B -d q4_0 -n 1 -i 50 | grep step
  LAMM_GEMV_VARIANT=$v timeout -k 10 120 $B -d q4_0 -n 1 -i 50 --batch-proj | grep step
done
