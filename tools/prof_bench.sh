# Full GPU test suite, the default bench line, and the rocprofv3 kernel statistics of the
# same bench command (profiles/ copies are made by hand afterwards).  Run via gpurun.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1
timeout -k 10 400 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rm -rf gpurun_out/prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 -u bench.py --no-cpu --no-llama > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err
