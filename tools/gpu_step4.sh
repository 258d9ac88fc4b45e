# GPU step (via gpurun): the llama.cpp parity tests (2-layer modes, nodes, 32 layers), then the
# float-order modes end to end and the reference-order kernel timings under the tracer.
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/g5}
mkdir -p "$OUT"
timeout -k 10 1000 python -u -m pytest tests/test_gpu_llama_e2e.py -x -v -s --timeout 400 --timeout-method thread > "$OUT/e2e.log" 2>&1
bash tools/gpu_e2e_modes.sh "$OUT/modes"
rm -rf "$OUT/rt_prof"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rt_prof" -o run -- python3 -u tools/ref_order_time.py > "$OUT/ref_time.log" 2>&1
