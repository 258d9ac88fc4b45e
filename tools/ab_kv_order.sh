# gemm_fp6_kv_kernel's per-unit issue order (F6_KV_ORDER builds of tools/prep_probe.hip: 0 production
# S, E/2, P, E/2; 1 P, E/2, S, E/2; 2 S, P, E), config 3 main kernel alone, twice each alternating.
# Build: for o in 0 1 2; do hipcc ... -DF6_KV_ORDER=$o ... -o tools/prep_probe_o$o; done (see prep_probe.hip)
# Usage (via gpurun): bash tools/ab_kv_order.sh gpurun_out/<dir>
set -e
OUT=${1:-gpurun_out/ab_kv_order}
mkdir -p "$OUT"
for r in 1 2; do
  for o in 0 1 2; do
    timeout -k 10 100 tools/prep_probe_o$o gemm_kvmain_p3 > "$OUT/o${o}_r$r.json"
  done
done
