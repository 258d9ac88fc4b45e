# fp6 GEMM K-group epilogue: C stores non-temporal (the default build, F6_C_NT=1) vs cached
# (VAR = build_var/liblamm_hip_c0.so, -DF6_C_NT=0).  Alternating processes of the whole-launch
# timing (ab_fp6_kgroups.py, automatic plan), REPS times.  (The first run compared a
# -DF6_C_NT=1 variant against the then-default cached build: profiles/r02/ab_c_nt/.)
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/c_nt}
REPS=${REPS:-3}
VAR=la-llama.cpp_amd/build_var/liblamm_hip_c0.so
mkdir -p "$OUT"
for rep in $(seq 1 $REPS); do
  ARMS=-1 timeout -k 10 200 python -u tools/ab_fp6_kgroups.py > "$OUT/ab_nt_$rep.log" 2>&1
  LAMM_HIP_LIB=$PWD/$VAR ARMS=-1 timeout -k 10 200 python -u tools/ab_fp6_kgroups.py > "$OUT/ab_cached_$rep.log" 2>&1
done
