# fused activation prep in the K-group fp6 GEMM: parity tests, then config-3 / Llama prefill timing
# A/B (whole launches, hipGraph) and the kernels' rocprof durations (run via gpurun)
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/fprep}
rm -rf "$OUT"; mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -k "fp6 or config3 or fuzz or f32_activations" > "$OUT/pytest.log" 2>&1
for fp in 1 0 1 0; do
  LAMM_FP6_FUSED_PREP=$fp ARMS=1 timeout -k 10 200 python -u tools/ab_fp6_kgroups.py >> "$OUT/kg_fp$fp.log" 2>&1
done
SPLITS=0 VARIANTS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d "$OUT/prof" -o run -- python3 -u tools/ab_fp6_single.py > "$OUT/prof.log" 2>&1
