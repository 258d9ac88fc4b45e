#!/bin/bash
# Config-2 issue modes (tools/measure_config2.py) untraced, then under the kernel tracer per phase.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/m2
timeout -k 10 240 python3 -u tools/measure_config2.py > gpurun_out/m2/plain.json 2> gpurun_out/m2/plain.err
for ph in spaced b2b cloop graph; do
  rm -rf gpurun_out/m2/prof_$ph
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/m2/prof_$ph -o run -- python3 -u tools/measure_config2.py --phase $ph > gpurun_out/m2/prof_$ph.json 2> gpurun_out/m2/prof_$ph.err
done
