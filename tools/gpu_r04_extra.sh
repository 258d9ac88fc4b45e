# Round-4 extras on one GPU: the bench's N>1 paths rehearsed at 2 / 4 / 8 ranks (gather bit-exact),
# then config 5 decode with each LAMM_HIP_HELPERS mode at -t 16 / -t 8
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r04_extra}
mkdir -p "$OUT"
bash tools/gpu_multirank.sh "$OUT/multirank"
timeout -k 10 900 python -u tools/e2e_helpers.py "$OUT/e2e_helpers.json" > "$OUT/e2e_helpers.log" 2>&1
