# dq16 with two waves per K-group (8 waves, 2 per SIMD) vs one: config 3 and config 4 shapes, parity
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/dq6}
mkdir -p "$OUT"
V=la-llama.cpp_amd/var_dq
for fmt in q4_0 q8_0 q5_1; do
for lib in la-llama.cpp_amd/liblamm_hip.so $V/liblamm_hip_dq_wh1.so $V/liblamm_hip_dq_wh2nbv2.so; do
  LAMM_HIP_LIB=$lib timeout -k 10 120 python -u tools/dq_ab.py $fmt >> "$OUT/ab.jsonl" 2>> "$OUT/ab.err"
done
done
LAMM_HIP_LIB=la-llama.cpp_amd/liblamm_hip.so timeout -k 10 120 python -u tools/dq_ab.py q4_0 4096 512 11008 >> "$OUT/ab.jsonl" 2>> "$OUT/ab.err"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "dq16 or config3" --timeout 300 --timeout-method thread > "$OUT/pytest_dq.log" 2>&1
