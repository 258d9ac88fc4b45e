# K-group fp6 GEMM (config 3 single slice) ablations under rocprofv3 kernel trace (run via gpurun)
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/abkg}
rm -rf "$OUT"; mkdir -p "$OUT"
SPLITS=0 VARIANTS=${VARIANTS:-0,1,2,3,4,6,7} timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d "$OUT" -o run -- python3 -u tools/ab_fp6_single.py > "$OUT/run.log" 2>&1
