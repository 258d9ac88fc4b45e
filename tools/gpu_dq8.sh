# dq16 v2: loads only at 1 / 2 quads in flight, unpack + MFMA only, production at 1 / 2 (config 3, q4_0)
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/dq8}
mkdir -p "$OUT"
V=la-llama.cpp_amd/var_dq
for rep in 1 2; do
for lib in la-llama.cpp_amd/liblamm_hip.so $V/liblamm_hip_dq_l1.so $V/liblamm_hip_dq_l2.so $V/liblamm_hip_dq_c1.so $V/liblamm_hip_dq_n2.so; do
  LAMM_HIP_LIB=$lib timeout -k 10 120 python -u tools/dq_ab.py q4_0 >> "$OUT/ab.jsonl" 2>> "$OUT/ab.err"
done
done
