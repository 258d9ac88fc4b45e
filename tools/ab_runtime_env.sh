# HIP runtime knobs on the Llama-7B decode step (launch-bound): kernel arguments in device
# memory, graph packet capture; profiles/r01/llama_runtime_env_ab.txt.  Run via gpurun.
set -e
B=./la-llama.cpp_amd/llama-matmul-bench
run() { echo "== $*"; env "$@" timeout -k 10 120 $B -d q4_0 -n 1 -i 100 | grep step | cut -c1-70; }
run X=0
run HIP_FORCE_DEV_KERNARG=1
run DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
run DEBUG_CLR_GRAPH_PACKET_CAPTURE=1
run X=0
