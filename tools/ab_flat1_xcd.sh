# XCD-aware row groups in gemv_flat1_kernel vs tools/_old (the commit before): GEMV parity tests,
# then config 2 through the library (probe "lib") 5 x alternating.  Usage: bash tools/ab_flat1_xcd.sh OUT
set -e
OUT=${1:-gpurun_out/ab_flat1_xcd}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "row_slab or row_per_wave or gemv or golden" --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
for i in 1 2 3 4 5; do
  echo "new $(timeout -k 10 60 tools/gemv_probe lib 2>/dev/null)" >> "$OUT/ab.txt"
  echo "old $(LD_LIBRARY_PATH=$PWD/tools/_old timeout -k 10 60 tools/gemv_probe lib 2>/dev/null)" >> "$OUT/ab.txt"
done
