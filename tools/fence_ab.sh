set -e
mkdir -p gpurun_out/fence
timeout -k 10 300 python -u tools/issue_modes.py > gpurun_out/fence/agent.jsonl 2> gpurun_out/fence/agent.err
LAMM_AQL_FENCE=none timeout -k 10 300 python -u tools/issue_modes.py > gpurun_out/fence/none.jsonl 2> gpurun_out/fence/none.err
