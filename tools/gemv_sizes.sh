# Single-call q4_0 decode GEMV at the Llama-7B projection sizes (q8 activations, one slice):
# per-launch us and TB/s of the library's default kernel.  Usage: bash tools/gemv_sizes.sh OUT
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/gemv_sizes}
mkdir -p "$OUT"
for mk in "4096 4096" "12288 4096" "22016 4096" "4096 11008" "11008 4096"; do
  set -- $mk
  timeout -k 10 120 python -u tools/bench_gemv_n.py q4_0 $1 $2 >> "$OUT/sizes.jsonl"
done
