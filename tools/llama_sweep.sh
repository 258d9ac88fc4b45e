# llama-matmul-bench (Llama-7B weight matmuls per step, hipGraph) for decode and prefill
# chunks; profiles/r01/llama_matmul_bench.txt.  Run via gpurun.
set -e
B=./la-llama.cpp_amd/llama-matmul-bench
timeout -k 10 120 $B -d q4_0 -n 1 -i 50
timeout -k 10 120 $B -d q4_0 -n 1 -i 50 --no-graph
timeout -k 10 120 $B -d q4_0 -n 8 -i 50
timeout -k 10 120 $B -d q4_0 -n 128 -i 10 -s
timeout -k 10 120 $B -d q4_0 -n 512 -i 5 -s
timeout -k 10 120 $B -d q4_k -n 1 -i 50 --output-type q6_k
timeout -k 10 120 $B -d q4_k -n 512 -i 5 -s
