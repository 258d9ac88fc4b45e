# A/B of the prefill engines and their K-split counts at la-benchmark-matmult's own shape
# (K=11008, M=4096, N=128); profiles/r01/ab_driver_split.txt.  Run via gpurun.
set -e
B=./la-llama.cpp_amd/la-benchmark-matmult
for d in q4_0 q5_1 q8_0; do
 for cfg in "i8:1::" "i8:::" "i8:8::" "i8:16::" "fp6::16:" "fp6::16:-s" "::::" "::::-s"; do
  IFS=: read path i8s f6s _ s <<< "$cfg"
  case $d in q5_1|q8_0) [ "$path" = fp6 ] && continue;; esac
  echo "== $d path=${path:-auto} i8split=${i8s:-auto} fp6split=${f6s:-auto} $s"
  LAMM_GEMM_PATH=$path LAMM_I8_SPLIT=$i8s LAMM_FP6_SPLIT=$f6s timeout -k 10 100 $B -d $d -t 16 -i 20 $s | grep -E "Average|ABORT"
 done
done
