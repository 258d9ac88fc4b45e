# Round rehearsal on one GPU, in one call: every -m gpu test (one process), smoke(), the
# default bench line, and the rocprofv3 kernel statistics of the bench's GPU legs (copied to
# profiles/ by hand afterwards); EXTRA (optional) = one more script to run after them.
# Usage (via gpurun): bash tools/gpu_round.sh gpurun_out/<dir> [extra.sh]
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/round}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1
timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
rm -rf "$OUT/prof"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 -u bench.py --no-cpu --no-llama > "$OUT/bench_prof.json" 2> "$OUT/bench_prof.err"
if [ -n "$2" ]; then bash "$2" "$OUT/extra"; fi
