# Probe builds of the reference-order kernels (ab_libs/liblamm_hip_ref_<name>.so): the library's
# objects with lamm_ref.hip recompiled under -D flags (ab_libs travels to the GPU box).
# Usage: bash tools/build_ref_var.sh name "-DREF_AB=1 ..."
set -e
cd "$(dirname "$0")/../la-llama.cpp_amd"
make -s liblamm_hip.so
mkdir -p ab_libs
NAME=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -mllvm -amdgpu-mfma-vgpr-form -fno-slp-vectorize $* -c csrc/lamm_ref.hip -o ab_libs/ref_$NAME.o
OBJS=$(ls build/*.o | grep -v lamm_ref.hip.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -o ab_libs/liblamm_hip_ref_$NAME.so $OBJS ab_libs/ref_$NAME.o -ldl
rm -f ab_libs/ref_$NAME.o
echo ab_libs/liblamm_hip_ref_$NAME.so
