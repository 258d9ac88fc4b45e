# plane-split fp6 activation prep (prep_b_fp6_hs) vs the one-thread-per-block prep: parity tests,
# interleaved whole-launch A/B (hipGraph), rocprof durations of both preps (run via gpurun)
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/prep_hs}
rm -rf "$OUT"; mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -k "fp6 or config3 or fuzz or f32_activations" > "$OUT/pytest.log" 2>&1
ABVAR=LAMM_PREP_HSPLIT ARMS=1,0 timeout -k 10 300 python -u tools/ab_fp6_kgroups.py > "$OUT/ab.log" 2>&1
for hs in 1 0; do
  LAMM_PREP_HSPLIT=$hs SPLITS=0 VARIANTS=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$OUT/prof_hs$hs" -o run -- python3 -u tools/ab_fp6_single.py > "$OUT/prof_hs$hs.log" 2>&1
done
