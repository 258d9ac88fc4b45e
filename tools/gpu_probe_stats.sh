# One GPU call: the GEMV probe (new library, previous library via tools/_old, a kernarg-preload
# build of the probe), every -m gpu test, then the config-5 boundary stats (tools/e2e_stats.sh).
# Usage (via gpurun): bash tools/gpu_probe_stats.sh
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/g1}
mkdir -p $OUT
timeout -k 10 150 tools/gemv_probe > $OUT/probe_new.json 2> $OUT/probe_new.err
LD_LIBRARY_PATH=$PWD/tools/_old timeout -k 10 60 tools/gemv_probe lib > $OUT/probe_oldlib.json 2>&1
timeout -k 10 150 tools/gemv_probe_pre > $OUT/probe_pre.json 2> $OUT/probe_pre.err
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
bash tools/e2e_stats.sh $OUT/stats
