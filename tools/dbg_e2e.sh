#!/bin/bash
# isolate config-5 parity differences: dump every F32 node of the prefill on both builds
OUT=gpurun_out/dbg
T=${TMPDIR:-/tmp}/dbg_e2e
mkdir -p $OUT $T/cpu $T/hip
M=$T/synth2.gguf
oracle/_ref/llama_e2e_lamm3 -m $M --layers 2 --write-only || exit 1
oracle/_ref/llama_e2e_lamm3 -m $M -t 8 -p ${P:-32} -n 0 --dump $T/cpu > /dev/null 2>&1 || exit 1
env "$@" integration/_build/llama_e2e_hip -m $M -t 8 -p ${P:-32} -n 0 --dump $T/hip > /dev/null 2>&1 || exit 1
python3 - $T > $OUT/nodes_${P:-32}.txt <<'PY'
import numpy as np, os, sys
T = sys.argv[1]
for f in sorted(os.listdir(T + "/cpu")):
    a = np.fromfile(f"{T}/cpu/{f}", np.float32)
    hp = f"{T}/hip/{f}"
    if not os.path.exists(hp):
        print(f, "missing in hip"); continue
    b = np.fromfile(hp, np.float32)
    d = np.abs(a - b).max() / (np.abs(a).max() + 1e-30)
    print(f"{f:60s} rel {d:.2e}  absmax {np.abs(a).max():.3e}")
PY
head -60 $OUT/nodes_${P:-32}.txt
