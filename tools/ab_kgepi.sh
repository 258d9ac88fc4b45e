# K-group fp6 GEMM epilogue: parity tests, then config-3 / Llama prefill timing (whole launches,
# hipGraph; tools/ab_fp6_kgroups.py) and the main kernel's rocprof duration (run via gpurun)
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/kgepi}
rm -rf "$OUT"; mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -k "fp6 or config3 or fuzz" > "$OUT/pytest.log" 2>&1
ARMS=0,1,2 timeout -k 10 300 python -u tools/ab_fp6_kgroups.py > "$OUT/kg.log" 2>&1
SPLITS=0 VARIANTS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d "$OUT/prof" -o run -- python3 -u tools/ab_fp6_single.py > "$OUT/prof.log" 2>&1
