#!/bin/bash
# HBM traffic of the config-2 single-call GEMV (gemv_rpw_kernel): two rocprofv3 --pmc passes
# (FETCH_SIZE, WRITE_SIZE), each its own run of tools/pmc_rpw.py.  FETCH_SIZE's scale for this
# kernel's access pattern (b128 + b64 loads at 4-byte offsets, MI355X_MICROARCH.md §HBM: only
# 16-B-per-lane streaming reads are calibrated) comes from the 33-slice launch of the same
# kernel in the same run: 312 MB no cache holds, read once.  Run via gpurun.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/pmc_rf gpurun_out/pmc_rw
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_rf -o f -- python3 tools/pmc_rpw.py > gpurun_out/pmc_rf.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_rw -o w -- python3 tools/pmc_rpw.py > gpurun_out/pmc_rw.log 2>&1
F=$(find gpurun_out/pmc_rf -name "*counter_collection.csv" | head -1)
W=$(find gpurun_out/pmc_rw -name "*counter_collection.csv" | head -1)
python3 tools/pmc_traffic_rpw.py "$F" "$W" gpurun_out/traffic_q4_0_gemv_single.json
