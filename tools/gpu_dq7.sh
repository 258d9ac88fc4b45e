# L2 behaviour of dq16 (config 3, q4_0): TCC hits / misses / read requests to memory, two passes
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/dq7}
mkdir -p "$OUT"
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$OUT/pmc_hit" -o run -- python3 tools/dq_ab.py q4_0 > "$OUT/pmc_hit.log" 2>&1
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_REQ_sum --output-format csv -d "$OUT/pmc_req" -o run -- python3 tools/dq_ab.py q4_0 > "$OUT/pmc_req.log" 2>&1
LAMM_GEMM_PATH=fp6 timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$OUT/pmc_hit_fp6" -o run -- python3 tools/bench_gemm_one.py q4_0 > "$OUT/pmc_hit_fp6.log" 2>&1 || true
