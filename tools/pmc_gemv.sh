# HBM traffic of the config-2 GEMV kernel: two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE),
# each its own run, then tools/pmc_traffic.py -> profiles/traffic_q4_0_gemv.json.  Run via gpurun.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/pmc_f gpurun_out/pmc_w
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_f -o f -- python3 bench.py --no-gemm --no-cpu --steps 10 --warmup 2 > gpurun_out/pmc_f.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_w -o w -- python3 bench.py --no-gemm --no-cpu --steps 10 --warmup 2 > gpurun_out/pmc_w.log 2>&1
F=$(find gpurun_out/pmc_f -name "*counter_collection.csv" | head -1)
W=$(find gpurun_out/pmc_w -name "*counter_collection.csv" | head -1)
python3 tools/pmc_traffic.py "$F" "$W" gemv_stream_dma_kernel gpurun_out/traffic_q4_0_gemv.json 312111360
