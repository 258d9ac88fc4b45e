# ggml-boundary end-to-end (PCIe included) with and without pinned host staging
# (LAMM_HIP_PINNED); the reference's unchanged ggml linked to liblamm_hip.so, 1 ggml thread.
set -e
X=oracle/_ref/ref_driver_hip
for pin in 0 1 0 1; do
  for shape in "4096 1 4096" "4096 8 4096" "4096 512 4096"; do
    echo "pinned=$pin $(LAMM_HIP_PINNED=$pin timeout -k 10 60 $X bench q4_0 $shape 1 100000 3)"
  done
done
