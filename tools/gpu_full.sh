# round-end rehearsal on one GPU: every -m gpu test (one process), smoke(), the default bench, the
# driver's own bench command (20 steps), and the rocprofv3 kernel statistics of the bench
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/full}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1
timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
if [ -n "$PROF" ]; then
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-llama --no-cpu > "$OUT/bench_driver_steps.json" 2> "$OUT/bench_driver_steps.err"
  rm -rf "$OUT/prof"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 -u bench.py --no-cpu --no-llama > "$OUT/bench_prof.json" 2> "$OUT/bench_prof.err"
fi
