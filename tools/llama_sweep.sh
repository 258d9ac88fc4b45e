# llama-matmul-bench (Llama-7B weight matmuls per step, hipGraph) for decode and prefill
# chunks, 7 launches per layer (as llama.cpp-b2430), --batch-proj (4 per layer) and
# --concurrent (7 per layer, wk/wv and ffn_up on forked graph branches);
# profiles/r01/llama_matmul_bench.txt.  Run via gpurun.
set -e
B=./la-llama.cpp_amd/llama-matmul-bench
for extra in "" "--batch-proj" "--concurrent"; do
  timeout -k 10 120 $B -d q4_0 -n 1 -i 50 $extra
  timeout -k 10 120 $B -d q4_0 -n 8 -i 50 $extra
  timeout -k 10 120 $B -d q4_0 -n 128 -i 10 -s $extra
  timeout -k 10 120 $B -d q4_0 -n 512 -i 5 -s $extra
  timeout -k 10 120 $B -d q4_k -n 1 -i 50 $extra
  timeout -k 10 120 $B -d q4_k -n 512 -i 5 -s $extra
done
