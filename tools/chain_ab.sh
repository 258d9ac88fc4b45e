# decode step through llama-matmul-bench: separate launches, --batch-proj, --chain (one launch)
set -e
B=./la-llama.cpp_amd/llama-matmul-bench
for mode in "" --batch-proj --chain; do
  echo "== $mode"
  timeout -k 10 120 $B -d q4_0 -n 1 -i 50 $mode | grep -v "^llama-matmul-bench"
done
