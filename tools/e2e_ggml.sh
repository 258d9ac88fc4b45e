# ggml-boundary end-to-end timings (PCIe included): the reference's unchanged ggml graph
# compute linked to liblamm_hip.so (oracle/_ref/ref_driver_hip), 1 ggml thread.  Run via gpurun.
set -e
mkdir -p gpurun_out
X=oracle/_ref/ref_driver_hip
: > gpurun_out/e2e.txt
for t in q4_0 q4_k q8_0; do
  for shape in "4096 1 4096" "4096 8 4096" "4096 512 4096"; do
    timeout -k 10 60 $X bench $t $shape 1 100000 3 >> gpurun_out/e2e.txt
  done
done
