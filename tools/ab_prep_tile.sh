# fp6 activation prep workgroup size (F6_PB_NB blocks per row: 8 production, 4, 2 -- 256 / 512 /
# 1024 workgroups for config 3) via variant libraries in tools/_var: parity of the fp6 GEMM with each,
# then the bench's config 3 lines, alternating.  Usage (via gpurun): bash tools/ab_prep_tile.sh OUT
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/ab_prep_tile}
mkdir -p "$OUT"
for v in 4 2; do
  LAMM_HIP_LIB=$PWD/tools/_var/liblamm_hip_pb$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "fp6 or config3 or gemm_q4" --timeout 300 --timeout-method thread > "$OUT/pytest_pb$v.log" 2>&1
done
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --no-llama --no-cpu --no-config1 --no-config4 > "$OUT/pb8_$i.json" 2>/dev/null
  for v in 4 2; do
    LAMM_HIP_LIB=$PWD/tools/_var/liblamm_hip_pb$v.so timeout -k 10 300 python -u bench.py --no-llama --no-cpu --no-config1 --no-config4 > "$OUT/pb${v}_$i.json" 2>/dev/null
  done
done
