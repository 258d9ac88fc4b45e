# Probe builds of the fp6 GEMM file (ab_libs/liblamm_hip_fp6_<name>.so): the library's objects with
# lamm_gemm_fp6.hip recompiled under -D flags (ab_libs travels to the GPU box).
# Usage: bash tools/build_fp6_var.sh name "-DF6_PREP_AB=1 ..."
set -e
cd "$(dirname "$0")/../la-llama.cpp_amd"
make -s liblamm_hip.so
mkdir -p ab_libs
NAME=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -fno-slp-vectorize $* -c csrc/lamm_gemm_fp6.hip -o ab_libs/fp6_$NAME.o
OBJS=$(ls build/*.o | grep -v lamm_gemm_fp6.hip.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -o ab_libs/liblamm_hip_fp6_$NAME.so $OBJS ab_libs/fp6_$NAME.o -ldl -L/opt/rocm/lib -lhsa-runtime64
rm -f ab_libs/fp6_$NAME.o
echo ab_libs/liblamm_hip_fp6_$NAME.so
