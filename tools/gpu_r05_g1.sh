set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$PWD/la-llama.cpp_amd:$PWD/tests
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "dq16 or default_engine_range" tests/test_gpu_ref_order.py::test_reference_order_prefill_full_size tests/test_gpu_ggml_boundary.py::test_pool_jobs tests/test_gpu_ggml_boundary.py::test_boundary_prefill_value_range > gpurun_out/r05_g1_tests.log 2>&1 && \
timeout -k 10 400 python -u bench.py --no-llama --no-cpu --no-config1 > gpurun_out/r05_g1_bench.json 2> gpurun_out/r05_g1_bench.err
