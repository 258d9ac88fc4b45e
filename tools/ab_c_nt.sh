# fp6 GEMM K-group epilogue: C stores non-temporal (build_var/liblamm_hip_cnt.so, -DF6_C_NT=1)
# vs the default build.  Parity of the variant on the config-3 tests, then alternating
# processes of the whole-launch timing (ab_fp6_kgroups.py, K-group arm) and rocprof of each.
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/c_nt}
VAR=la-llama.cpp_amd/build_var/liblamm_hip_cnt.so
rm -rf "$OUT"; mkdir -p "$OUT"
LAMM_HIP_LIB=$PWD/$VAR timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -k "config3 or k_groups" > "$OUT/pytest_var.log" 2>&1
for rep in 1 2; do
  ARMS=-1 timeout -k 10 200 python -u tools/ab_fp6_kgroups.py > "$OUT/ab_default_$rep.log" 2>&1
  LAMM_HIP_LIB=$PWD/$VAR ARMS=-1 timeout -k 10 200 python -u tools/ab_fp6_kgroups.py > "$OUT/ab_cnt_$rep.log" 2>&1
done
SPLITS=0 VARIANTS=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
  -d "$OUT/prof_default" -o run -- python3 -u tools/ab_fp6_single.py > "$OUT/prof_default.log" 2>&1
LAMM_HIP_LIB=$PWD/$VAR SPLITS=0 VARIANTS=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
  -d "$OUT/prof_cnt" -o run -- python3 -u tools/ab_fp6_single.py > "$OUT/prof_cnt.log" 2>&1
