# decode-step GEMV A/B on the Llama-7B weight-matmul step (llama-matmul-bench, hipGraph):
# one launch per projection vs --batch-proj (q|k|v and gate|up as one launch each), across
# the decode GEMV choices LAMM_GEMV_RPW (unset = default policy, 0 = wave-group kernels,
# n = row-per-wave kernel with n waves per workgroup).
set -e
B=./la-llama.cpp_amd/llama-matmul-bench
for v in default 0 4 8 16; do
  for bp in "" --batch-proj; do
    echo "== LAMM_GEMV_RPW=$v $bp"
    if [ "$v" = default ]; then
      timeout -k 10 120 $B -d q4_0 -n 1 -i 50 $bp | grep step
    else
      LAMM_GEMV_RPW=$v timeout -k 10 120 $B -d q4_0 -n 1 -i 50 $bp | grep step
    fi
  done
done
