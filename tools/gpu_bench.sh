# The driver's bench command, plain, then under the kernel tracer (via gpurun).
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/bench}
mkdir -p "$OUT"
rm -rf "$OUT/prof"
timeout -k 10 600 python3 -u bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 -u bench.py --steps 20 --warmup 5 --no-cpu --no-llama > "$OUT/bench_under_rocprof.json" 2> "$OUT/bench_under_rocprof.err"
