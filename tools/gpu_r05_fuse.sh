# round 5: fp6 K-group kernel with the activation prep fused in -- bit identity, config 3 timing, trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$PWD/la-llama.cpp_amd:$PWD/tests
O=gpurun_out/r05_fuse
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "fused_prep or config3" > $O/tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-llama --no-cpu --no-config1 --no-config4 --steps 200 > $O/bench_fused.json 2> $O/bench_fused.err && \
LAMM_FP6_FUSE=0 timeout -k 10 300 python -u bench.py --no-llama --no-cpu --no-config1 --no-config4 --steps 200 > $O/bench_unfused.json 2> $O/bench_unfused.err && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --no-llama --no-cpu --no-config1 --no-config4 --steps 50 > $O/prof.log 2>&1
