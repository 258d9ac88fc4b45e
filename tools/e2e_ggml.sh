set -e
X=oracle/_ref/ref_driver_hip
for q in 1 0; do
  for shape in "4096 1 4096" "4096 512 4096" "4096 8 4096"; do
    echo "gpu_quant=$q $shape" >> gpurun_out/e2e.txt
    LAMM_HIP_GPU_QUANT=$q timeout -k 10 60 $X bench q4_0 $shape 1 100000 3 >> gpurun_out/e2e.txt
  done
done
