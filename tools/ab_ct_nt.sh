# fp6 GEMM whole-tile (KG = 1, 256x128 tiles: batched slices, split-K partials) epilogue stores
# (first run, before non-temporal became the default; VAR then = the -DF6_CT_NT=1 build):
# non-temporal (VAR = build_var/liblamm_hip_ctnt.so, -DF6_CT_NT=1) vs the default cached stores.
# Parity of the variant on the fp6 / config-3 tests, then alternating processes of the
# whole-launch timing (ab_fp6_kgroups.py, automatic plan), REPS times.
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/ct_nt}
REPS=${REPS:-3}
VAR=la-llama.cpp_amd/build_var/liblamm_hip_ctnt.so
mkdir -p "$OUT"
LAMM_HIP_LIB=$PWD/$VAR timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -k "fp6 or config3" > "$OUT/pytest_var.log" 2>&1
for rep in $(seq 1 $REPS); do
  SHAPES=config3_4slices,config3_1slice ARMS=-1 timeout -k 10 200 python -u tools/ab_fp6_kgroups.py > "$OUT/ab_default_$rep.log" 2>&1
  LAMM_HIP_LIB=$PWD/$VAR SHAPES=config3_4slices,config3_1slice ARMS=-1 timeout -k 10 200 python -u tools/ab_fp6_kgroups.py > "$OUT/ab_ctnt_$rep.log" 2>&1
done
