# Probe builds of the dq16 GEMM (var_dq/liblamm_hip_dq_<name>.so): the library's objects with
# lamm_gemm_dq.hip recompiled under -D flags.  Usage: bash tools/build_dq_var.sh name "-DDQ_AB=1 ..."
set -e
cd "$(dirname "$0")/../la-llama.cpp_amd"
make -s liblamm_hip.so
mkdir -p var_dq
NAME=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result $* -c csrc/lamm_gemm_dq.hip -o var_dq/dq_$NAME.o
OBJS=$(ls build/*.o | grep -v lamm_gemm_dq.hip.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -o var_dq/liblamm_hip_dq_$NAME.so $OBJS var_dq/dq_$NAME.o -ldl
echo var_dq/liblamm_hip_dq_$NAME.so
