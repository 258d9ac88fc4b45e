# la-benchmark-matmult over every weight type at its default shape (K=11008, M=4096, N=128),
# plain and weight-stationary (-s); profiles/r01/driver_sweep.txt.  Run via gpurun.
set -e
B=./la-llama.cpp_amd/la-benchmark-matmult
for d in q4_0 q4_1 q5_0 q5_1 q8_0 q2_k q4_k q5_k q6_k f16 f32; do
  for s in "" "-s"; do
    echo "== $d $s"
    timeout -k 10 100 $B -d $d -t 16 -i 20 $s | grep -E "Average|weights:|ABORT"
  done
done
